# Sub-batch count sweep (interleaved): tools/split_sweep.sh <tag> <config> <rounds> <split>...
set -e
TAG=$1; CFG=$2; R=$3; shift 3
OUT=gpurun_out/split_${TAG}.txt
: > "$OUT"
for r in $(seq 1 "$R"); do
  for s in "$@"; do
    timeout -k 10 180 python3 bench.py --config "$CFG" --split "$s" --extras none --no-cpu-baseline --steps 60 --warmup 5 \
      > gpurun_out/split_${TAG}_last.json 2>/dev/null
    python3 -c "
import json; d=json.loads(open('gpurun_out/split_${TAG}_last.json').read().strip().splitlines()[-1])
line='$CFG split=$s ms=%.4f step_frac=%.3f copy=%s' % (d['ms_per_step'], d['step_roofline']['frac'], d['box']['copy_GBps'])
print(line); open('$OUT','a').write(line+'\n')"
  done
done
