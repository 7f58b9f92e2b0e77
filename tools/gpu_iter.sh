#!/bin/bash
# One optimisation iteration on the GPU box: encode/decode parity tests, the default bench twice, and a
# short kernel trace with the last dispatches dumped (start/end/queue) to see the step's idle phases.
#   tools/gpu_iter.sh <tag>
set -e
TAG=${1:-it}
O=gpurun_out/iter_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q -m gpu \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python tools/stage_probe.py > $O/stage_probe.json 2>&1
for i in 1 2; do
  timeout -k 10 120 python bench.py --no-cpu-baseline > $O/bench$i.json 2> $O/bench$i.err
done
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/trace -o run --output-format csv \
  -- python3 bench.py --steps 6 --warmup 2 --no-cpu-baseline > $O/bench_trace.json 2> $O/trace.err
python3 tools/timeline.py $O/trace --group 2 --last-frac 0.3 --dump 40 > $O/timeline.txt
rm -rf $O/trace
