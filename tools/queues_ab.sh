#!/bin/bash
# C3 bench lines across HIP hardware-queue counts (GPU_MAX_HW_QUEUES), sub-batch counts and the per-plan
# small-segment side stream (--fork). tools/queues_ab.sh
set -e
export TMPDIR=/tmp
for q in 4 8; do for sp in 2 3 4; do for fk in "" "--fork"; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 120 python bench.py --no-cpu-baseline --extras none --split $sp $fk \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('queues $q split $sp fork=${fk:-no}', d['value'], d['ms_per_step'])"
done; done; done
