#!/bin/bash
# Batch k_scan knobs re-checked at the session-2 decode and small-segment limit.
set -e
O=gpurun_out/r03am
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
V="scan_w4 scan_nb2 scan_xcd"
COALAC_LIB=$L/scan_xcd.so timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  for c in C3 C2; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    for v in $V; do
      COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B --config $c > $O/${c}_${v}_$i.json 2>>$O/err.log
    done
  done
done
for f in $O/C*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
