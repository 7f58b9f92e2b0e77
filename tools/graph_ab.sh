#!/bin/bash
# Latency-bound configs: eager steps vs hipGraph replay with 1 / 4 / 10 steps per graph launch.
set -e
export TMPDIR=/tmp
for m in "off 1" "auto 1" "auto 4" "auto 10" "off 1" "auto 4"; do
  set -- $m
  timeout -k 10 200 python bench.py --config single --extras single_x2,C5 --no-cpu-baseline --graph $1 --graph-steps $2 \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('graph=$1 steps/graph=$2', 'single', d['value'], d['ms_per_step'], {k: (v['value'], v['ms_per_step']) for k, v in d['configs'].items()})"
done
