#!/bin/bash
# Staggered sub-batch scans (SplitPipeline stagger) vs free-running sub-batches: parity, then C3 / C2 / C4.
set -e
O=gpurun_out/r03v
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  for st in off on; do
    timeout -k 10 120 python bench.py $B --stagger $st > $O/c3_${st}_$i.json 2>>$O/err.log
    timeout -k 10 120 python bench.py $B --config C2 --stagger $st > $O/c2_${st}_$i.json 2>>$O/err.log
  done
done
for st in off on; do
  timeout -k 10 120 python bench.py $B --config C4 --stagger $st > $O/c4_${st}.json 2>>$O/err.log
  timeout -k 10 120 python bench.py $B --split 3 --stagger $st > $O/c3s3_${st}.json 2>>$O/err.log
  timeout -k 10 120 python bench.py $B --split 4 --stagger $st > $O/c3s4_${st}.json 2>>$O/err.log
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'], d.get('stagger'))"); done
