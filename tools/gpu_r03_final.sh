#!/bin/bash
# Session-2 final check at HEAD: GPU suite, smoke, the default bench line (all extras), a 2-rank gloo rehearsal
# of the self-launching multi-GPU path on this one GPU, and the aggregate tool.
set -e
O=gpurun_out/r03_final
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("C3", d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["traffic"])
for k, v in d["configs"].items():
    print(k, v["value"], v.get("ms_per_step", v.get("ms_per_client")), v["step_roofline"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
COALA_BENCH_DIST_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --extras none --no-cpu-baseline > $O/bench_g2.json 2> $O/bench_g2.err \
  || { tail -20 $O/bench_g2.err; exit 1; }
python -c "import json; d=json.load(open('$O/bench_g2.json')); print('gpus2', d['n_gpus'], d['value'], d['ms_per_step'], d['config']['parallelism'])"
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg.json 2>&1
tail -1 $O/agg.json | cut -c1-300
