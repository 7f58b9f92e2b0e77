#!/bin/bash
# k_aggregate with the base in the LDS tile (x = a + d, 2 ops per element and client): parity of the default
# build and its AGG_DEPTH / AGG_SPLIT variants, then tools/bench_aggregate.py against HEAD's kernel.
set -e
O=gpurun_out/r03t
mkdir -p $O
export TMPDIR=/tmp
T="tests/test_gpu_aggregate.py tests/test_reference_fixture.py tests/test_gpu_plugin.py"
timeout -k 10 300 python -u -m pytest $T -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
echo default; tail -1 $O/pytest.log
for v in agg_d8 agg_s4d8; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_new_$i.json 2>&1
  for v in agg_head agg_d8 agg_s4d8; do
    COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/${v}_$i.json 2>&1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03t/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["k_aggregate_ms"], d["roofline"]["frac"], d["ms"])
PY
