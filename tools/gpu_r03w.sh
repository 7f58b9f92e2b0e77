#!/bin/bash
# Two batches in flight (bench --inflight 2: consecutive steps on disjoint pooled streams and buffers) vs one.
set -e
O=gpurun_out/r03w
mkdir -p $O
export TMPDIR=/tmp
B="--extras none --no-cpu-baseline"
for i in 1 2; do
  for cfg in C3 C2 C4; do
    for inf in 1 2; do
      for sp in 1 2; do
        timeout -k 10 120 python bench.py $B --config $cfg --inflight $inf --split $sp > $O/${cfg}_i${inf}_s${sp}_$i.json 2>>$O/err.log
      done
    done
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
