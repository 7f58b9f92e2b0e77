#!/bin/bash
# Profiles at the session-2 decode (tools/profile_round.sh r03b), then C2 with 2 vs 3 sub-batches.
set -e
O=gpurun_out/r03ac
mkdir -p $O
export TMPDIR=/tmp
bash tools/profile_round.sh r03b > $O/profile.log 2>&1 || { tail -30 $O/profile.log; exit 1; }
tail -3 $O/profile.log
B="--extras none --no-cpu-baseline --config C2"
for i in 1 2; do
  for sp in 2 3; do
    timeout -k 10 120 python bench.py $B --split $sp > $O/c2_s${sp}_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
