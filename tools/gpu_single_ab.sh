#!/bin/bash
# Single-update A/B on the GPU box: GPU tests, then the 'single' config under each decode-prefill mode and
# the default bench line. tools/gpu_single_ab.sh <tag> [pytest selection]
set -e
TAG=${1:-single}
SEL=${2:-tests}
O=gpurun_out/single_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
for pf in ${PF:-none start scan small none start scan small}; do
  timeout -k 10 120 python bench.py --config single --extras none --no-cpu-baseline --steps 200 --warmup 20 \
    --prefill $pf >> $O/single_$pf.jsonl 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
done
timeout -k 10 300 python bench.py --no-cpu-baseline --extras none > $O/bench.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/single_*/single_*.jsonl")):
    for l in open(f):
        d = json.loads(l)
        print(f.split("/")[-1], d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["stages_ms"])
PY
cat $O/bench.json | cut -c1-400
