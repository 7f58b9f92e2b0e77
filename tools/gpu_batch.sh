#!/bin/bash
# One GPU-box session: decode ablation, GPU parity tests, select stamps, 1/16-client bench, and
# optionally (PROFILE=tag) the rocprof passes + host-inclusive rate. Every GPU step has its own time
# limit and the chain stops at the first failure.
set -e
export TMPDIR=/tmp
timeout -k 10 120 ./tools/decode_ablate > gpurun_out/decode_ablate.log 2>&1
timeout -k 10 480 python -m pytest tests/test_gpu_parity.py tests/test_gpu_aggregate.py -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1
timeout -k 10 120 python tools/select_stamps.py 16 > gpurun_out/stamps16.log 2>&1
for C in 1 16; do
  timeout -k 10 100 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --clients $C > gpurun_out/b_c${C}_f0.log 2>&1
done
if [ -n "$PROFILE" ]; then
  bash tools/profile_round.sh "$PROFILE"
  timeout -k 10 200 python tools/host_rate.py > gpurun_out/prof_$PROFILE/host_rate.jsonl 2> gpurun_out/prof_$PROFILE/host_rate.err
fi
timeout -k 10 120 python tools/bench_aggregate.py > gpurun_out/bench_aggregate.log 2>&1
