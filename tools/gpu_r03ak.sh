#!/bin/bash
# Batch plans: small-segment limit (segments encoded whole by one block) 4096 (default) vs 2048 / 1024.
set -e
O=gpurun_out/r03ak
mkdir -p $O
export TMPDIR=/tmp
COALAC_SMALL_MAX=1024 timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  for c in C3 C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_4096_$i.json 2>>$O/err.log
    COALAC_SMALL_MAX=2048 timeout -k 10 120 python bench.py $B --config $c > $O/${c}_2048_$i.json 2>>$O/err.log
    COALAC_SMALL_MAX=1024 timeout -k 10 120 python bench.py $B --config $c > $O/${c}_1024_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
