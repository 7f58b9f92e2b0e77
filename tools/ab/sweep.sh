set -e
O=gpurun_out/sweep; mkdir -p $O
for cfg in "16 2 1" "16 3 1" "16 4 1" "16 2 2" "16 1 2" "1 1 1" "1 1 2" "1 1 3" "1 1 4"; do set -- $cfg
  timeout -k 10 100 python bench.py --clients $1 --split $2 --inflight $3 --steps 40 --no-cpu-baseline > $O/c$1_s$2_i$3.json 2>&1; done
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['stages_ms'],d['step_roofline']['frac'])"; done
