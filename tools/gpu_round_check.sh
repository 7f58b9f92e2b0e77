#!/bin/bash
# Round check on the GPU box: GPU tests (one process), smoke(), the default bench line (all extras), and
# a 300-step single-update line. tools/gpu_round_check.sh <tag>
set -e
TAG=${1:-r02}
O=gpurun_out/rc_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("C3", d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["configs"].items():
    print(k, v["value"], v.get("ms_per_step", v.get("ms_per_client")), v["step_roofline"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
timeout -k 10 120 python bench.py --config single --extras none --no-cpu-baseline --steps 300 --warmup 20 \
  > $O/single.json 2>> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python -c "import json,sys; d=json.load(open('$O/single.json')); print('single', d['value'], d['ms_per_step'])"
