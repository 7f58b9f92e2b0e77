#!/bin/bash
# k_scan row compaction from the compares' scalar masks, staged rows without per-record overflow branches
# (variant scanrow) vs HEAD: parity, then C3 / C2 / C4 / single interleaved.
set -e
O=gpurun_out/r03af
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
COALAC_LIB=$L/scanrow.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py \
  tests/test_gpu_fullsize.py tests/test_gpu_mixed.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  for c in C3 C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    COALAC_LIB=$L/scanrow.so timeout -k 10 120 python bench.py $B --config $c > $O/${c}_scanrow_$i.json 2>>$O/err.log
  done
  timeout -k 10 120 python bench.py $B --config single --steps 300 > $O/single_def_$i.json 2>>$O/err.log
  COALAC_LIB=$L/scanrow.so timeout -k 10 120 python bench.py $B --config single --steps 300 > $O/single_scanrow_$i.json 2>>$O/err.log
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
