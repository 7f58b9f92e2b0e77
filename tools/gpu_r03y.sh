#!/bin/bash
# k_decode_lds 8-row passes, one unit per wave (dq8d1) and neighbours; weights and delta mode; C2 / C4.
set -e
O=gpurun_out/r03y
mkdir -p $O
export TMPDIR=/tmp
for v in dq8d1 dq8d1b8n; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py \
    tests/test_gpu_pipeline.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > $O/pytest_$v.log 2>&1 \
    || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
B="--extras none --no-cpu-baseline"
L=coala_amd/lib/variants
for i in 1 2; do
  timeout -k 10 120 python bench.py $B > $O/c3_def_$i.json 2>>$O/err.log
  for v in dq8d1 dq8d1x0 dq8d1s0 dq4d1; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B > $O/c3_${v}_$i.json 2>>$O/err.log
  done
  timeout -k 10 120 python bench.py $B --mode delta > $O/c3delta_def_$i.json 2>>$O/err.log
  for v in dq8d1 dq8d1b8n; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B --mode delta > $O/c3delta_${v}_$i.json 2>>$O/err.log
  done
  for c in C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    COALAC_LIB=$L/dq8d1.so timeout -k 10 120 python bench.py $B --config $c > $O/${c}_dq8d1_$i.json 2>>$O/err.log
  done
done
for sp in 1 3; do
  COALAC_LIB=$L/dq8d1.so timeout -k 10 120 python bench.py $B --split $sp > $O/c3s${sp}_dq8d1.json 2>>$O/err.log
  COALAC_LIB=$L/dq8d1.so timeout -k 10 120 python bench.py $B --config C2 --split $sp > $O/C2s${sp}_dq8d1.json 2>>$O/err.log
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
