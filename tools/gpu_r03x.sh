#!/bin/bash
# k_decode_lds weights mode: 8-row tile passes (2 LDS round trips per unit instead of 4) vs 4-row.
set -e
O=gpurun_out/r03x
mkdir -p $O
export TMPDIR=/tmp
COALAC_LIB=coala_amd/lib/variants/dq8.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
  -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $O/c3_def_$i.json 2>>$O/err.log
  for v in dq8 dq8d1 dq8d4; do
    COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python bench.py $B > $O/c3_${v}_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
