#!/bin/bash
# A/B of libcoalac.so (new, in tree) against tools/ab/libcoalac_old.so on the default bench; 2 runs each.
set -e
O=gpurun_out/ab; mkdir -p $O
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/new_$r.json 2>$O/new.err
done
cp coala_amd/lib/libcoalac.so /tmp/new.so; cp tools/ab/libcoalac_old.so coala_amd/lib/libcoalac.so
for r in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/old_$r.json 2>$O/old.err
done
cp /tmp/new.so coala_amd/lib/libcoalac.so
for f in $O/*.json; do python3 -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f',d['value'],d['ms_per_step'],d['stages_ms'])"; done
