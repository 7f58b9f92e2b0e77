#!/bin/bash
# Batch-config A/B of the library variants under coala_amd/lib/variants: C3 (twice), C2 and C4 bench lines.
#   tools/variant_ab.sh <tag> bash tools/batch_ab.sh
set -e
export TMPDIR=/tmp
for c in C3 C3 C2 C4; do
  timeout -k 10 120 python bench.py --no-cpu-baseline --extras none --config $c --steps 10 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('$c', d['value'], d['ms_per_step'])"
done
