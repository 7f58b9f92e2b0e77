#!/bin/bash
# Profile the default bench workload on the GPU box (run through gpurun from the repo root):
#   tools/profile_round.sh r03
# Pass 1: kernel trace + stats of the headline (C3 per GPU; per-kernel average durations, must agree with
# bench.py's HIP events). Pass 2: the same for the single-update config (inputs rotated over 3 buffer sets).
# Passes 3-6: FETCH_SIZE and WRITE_SIZE, in separate passes (they do not fit one TCC pass on gfx950), of the
# headline and of the single config; no trace domain besides the kernel trace. Summaries land in
# gpurun_out/prof_<tag>/.
set -e
TAG=${1:-r03}
OUT=gpurun_out/prof_${TAG}
mkdir -p "$OUT"
export TMPDIR=/tmp
B="--no-cpu-baseline --extras none"
S="--config single --graph off"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/trace" -o run --output-format csv \
  -- python3 bench.py --steps 10 --warmup 3 $B > "$OUT/bench_trace.json" 2> "$OUT/trace.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/single" -o run --output-format csv \
  -- python3 bench.py --steps 30 --warmup 3 $B --config single > "$OUT/bench_single.json" 2> "$OUT/single.err"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/fetch" -o run --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 $B > "$OUT/bench_fetch.json" 2> "$OUT/fetch.err"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/write" -o run --output-format csv \
  -- python3 bench.py --steps 3 --warmup 1 $B > "$OUT/bench_write.json" 2> "$OUT/write.err"
timeout -k 10 240 rocprofv3 --pmc FETCH_SIZE -d "$OUT/single_fetch" -o run --output-format csv \
  -- python3 bench.py --steps 6 --warmup 3 $B $S > "$OUT/bench_single_fetch.json" 2> "$OUT/single_fetch.err"
timeout -k 10 240 rocprofv3 --pmc WRITE_SIZE -d "$OUT/single_write" -o run --output-format csv \
  -- python3 bench.py --steps 6 --warmup 3 $B $S > "$OUT/bench_single_write.json" 2> "$OUT/single_write.err"
timeout -k 10 240 rocprofv3 --kernel-trace --stats -d "$OUT/agg" -o run --output-format csv \
  -- python3 tools/bench_aggregate.py > "$OUT/bench_aggregate_trace.json" 2> "$OUT/agg.err"
timeout -k 10 120 python3 tools/bench_aggregate.py > "$OUT/bench_aggregate.json" 2>> "$OUT/agg.err"
python3 tools/pmc_summary.py "$OUT" > "$OUT/summary.json"
mkdir -p "$OUT/s"
ln -s ../single "$OUT/s/trace"; ln -s ../single_fetch "$OUT/s/fetch"; ln -s ../single_write "$OUT/s/write"
python3 tools/pmc_summary.py "$OUT/s" > "$OUT/summary_single.json"
rm -rf "$OUT/s"
# bench --split 2 (default): its 8 joined roofline steps (the last groups) launch the two sub-batches' kernels together; the bench
# times their union interval, which this reproduces from the trace
python3 tools/timeline.py "$OUT/trace" --group 2 --last-groups 8 > "$OUT/timeline_union.json"
find "$OUT/trace" -name "*kernel_stats.csv" -exec python3 tools/filter_stats.py {} "$OUT/kernel_stats_codec.csv" \;
find "$OUT/single" -name "*kernel_stats.csv" -exec python3 tools/filter_stats.py {} "$OUT/kernel_stats_single.csv" \;
find "$OUT/agg" -name "*kernel_stats.csv" -exec python3 tools/filter_stats.py {} "$OUT/kernel_stats_aggregate.csv" \;
# keep the small summaries only (raw per-dispatch CSVs can exceed gpurun's 64 MiB pull limit)
du -sh "$OUT"/trace "$OUT"/single "$OUT"/fetch "$OUT"/write "$OUT"/agg || true
for s in trace single fetch write single_fetch single_write; do
  find "$OUT/$s" -name '*kernel_stats.csv' -exec cp {} "$OUT/${s}_kernel_stats.csv" \; || true
done
rm -rf "$OUT/trace" "$OUT/single" "$OUT/fetch" "$OUT/write" "$OUT/single_fetch" "$OUT/single_write" "$OUT/agg"
ls -la "$OUT"
