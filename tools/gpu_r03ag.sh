#!/bin/bash
set -e
O=gpurun_out/r03ag
mkdir -p $O
export TMPDIR=/tmp
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
  for c in C3 C2 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_def_$i.json 2>>$O/err.log
    PROBE_BOUNDS_DONE=1 timeout -k 10 120 python bench.py $B --config $c > $O/${c}_bdone_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
