set -e
O=gpurun_out/inf; mkdir -p $O
for C in 1 4; do for S in 1 2 3 4; do timeout -k 10 100 python bench.py --clients $C --steps 60 --warmup 5 --inflight $S --no-cpu-baseline > $O/c${C}_s$S.json 2>&1; done; done
for S in 1 2; do timeout -k 10 100 python bench.py --steps 20 --inflight $S --no-cpu-baseline > $O/c16_s$S.json 2>&1; done
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['stages_ms'])"; done
