#!/bin/bash
# Batch select-chain knobs re-tuned at the session-2 decode: k_emit units per wave, select group size.
set -e
O=gpurun_out/r03ad
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
for v in gu16 gu64; do
  COALAC_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
B="--extras none --no-cpu-baseline"
for i in 1 2; do
  for c in C3 C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    for v in emit2 emit4 gu16 gu64; do
      COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B --config $c > $O/${c}_${v}_$i.json 2>>$O/err.log
    done
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
