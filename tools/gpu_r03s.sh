#!/bin/bash
# Round-3 session 2: round check at HEAD + k_agg_blk A/B (parity of both variants, tools/bench_aggregate.py).
set -e
O=gpurun_out/r03s
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for v in agg_blk2 agg_blk4; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
for i in 1 2; do
  timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_base_$i.json 2>&1
  for v in agg_blk2 agg_blk4; do
    COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/${v}_$i.json 2>&1
  done
done
for f in $O/agg*.json; do echo $f; tail -1 $f | cut -c1-400; done
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("C3", d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["configs"].items():
    print(k, v["value"], v.get("ms_per_step", v.get("ms_per_client")), v["step_roofline"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
