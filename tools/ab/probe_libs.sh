#!/bin/bash
# Stage probe for each tools/ab/lib_*.so swapped in as coala_amd/lib/libcoalac.so.
set -e
O=gpurun_out/ab; mkdir -p $O
cp coala_amd/lib/libcoalac.so /tmp/keep.so
for L in tools/ab/lib_*.so; do
  n=$(basename $L .so)
  cp $L coala_amd/lib/libcoalac.so
  timeout -k 10 100 python tools/stage_probe.py > $O/$n.json 2>$O/$n.err
  python3 -c "import json;d=json.load(open('$O/$n.json'));print('$n',{k:d[k]['ms'] for k in ('scan_only_b2b','decode_only_b2b','step')})"
done
cp /tmp/keep.so coala_amd/lib/libcoalac.so
