#!/bin/bash
# Probe: C3 with the dense output buffer placed at an offset inside its allocation (decode-rate bimodality).
set -e
O=gpurun_out/r03an
mkdir -p $O
export TMPDIR=/tmp
B="--extras none --no-cpu-baseline"
for i in 1 2; do
  for kb in 0 4 64 1024 2112; do
    PROBE_OUT_OFFSET_KB=$kb timeout -k 10 120 python bench.py $B > $O/c3_off${kb}_$i.json 2>>$O/err.log
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
