#!/bin/bash
# k_decode_lds whole-unit passes (16 rows, one LDS round trip per unit) at 2 / 3 / 4 waves per block vs the
# 8-row default; C2 / C4 for the best.
set -e
O=gpurun_out/r03aa
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
COALAC_LIB=$L/dq16n128.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
  tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  timeout -k 10 120 python bench.py $B > $O/c3_def_$i.json 2>>$O/err.log
  for v in dq16n128 dq16n192 dq16n256 dq16n128x0; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B > $O/c3_${v}_$i.json 2>>$O/err.log
  done
done
for i in 1 2; do
  for c in C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    COALAC_LIB=$L/dq16n128.so timeout -k 10 120 python bench.py $B --config $c > $O/${c}_dq16n128_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
