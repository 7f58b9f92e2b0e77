#!/bin/bash
# k_aggregate_bg (base as the tile background, register-lean) at 4-5 waves per SIMD vs k_aggregate.
set -e
O=gpurun_out/r03ai
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
for v in bg_d8 bg_s4d8 bg_s4d16 bg_s4d4; do
  COALAC_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -q --timeout 120 \
    --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
for i in 1 2 3; do
  timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_def_$i.json 2>&1
  for v in bg_d8 bg_s4d8 bg_s4d16 bg_s4d4; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_${v}_$i.json 2>&1
  done
done
python - <<'PY'
import json, glob
for f in sorted(glob.glob("gpurun_out/r03ai/*.json")):
    d = json.loads(open(f).read().strip().splitlines()[-1])
    print(f.split("/")[-1], d["k_aggregate_ms"], d["roofline"]["frac"], d["ms"])
PY
