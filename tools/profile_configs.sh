#!/bin/bash
# Kernel trace + stats of bench configs, one rocprofv3 pass each (run through gpurun from the repo root):
#   tools/profile_configs.sh <tag> <config> [<config> ...]
# Summaries: gpurun_out/profc_<tag>/<config>_kernel_stats.csv (+ the bench line run under the profiler;
# KEEP_TRACE=1 also keeps <config>_kernel_trace.csv).
set -e
TAG=$1; shift
OUT=gpurun_out/profc_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
for C in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$C" -o run --output-format csv \
    -- python3 bench.py --config "$C" --extras none --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/${C}_bench.json" 2> "$OUT/${C}.err"
  find "$OUT/$C" -name '*kernel_stats.csv' -exec cp {} "$OUT/${C}_kernel_stats.csv" \;
  if [ -n "$KEEP_TRACE" ]; then find "$OUT/$C" -name '*kernel_trace.csv' -exec cp {} "$OUT/${C}_kernel_trace.csv" \; ; fi
  rm -rf "$OUT/$C"
done
ls -la "$OUT"
