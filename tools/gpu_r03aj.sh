#!/bin/bash
# single update: small segments in k_presel and the streaming k_scan at 7-8 blocks per CU (one wave generation)
# vs the small segments in k_scan's first blocks at 6 blocks per CU.
set -e
O=gpurun_out/r03aj
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
V="lat_ns7 lat_ns8 lat_ns8n4"
for v in $V; do
  COALAC_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
B="--extras none --no-cpu-baseline --steps 300 --warmup 20"
for i in 1 2 3 4; do
  timeout -k 10 120 python bench.py $B --config single > $O/single_def_$i.json 2>>$O/err.log
  timeout -k 10 120 python bench.py $B --config C5 > $O/c5_def_$i.json 2>>$O/err.log
  for v in $V; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B --config single > $O/single_${v}_$i.json 2>>$O/err.log
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B --config C5 > $O/c5_${v}_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
