# rocprof kernel stats of configs run as ONE sub-batch (no concurrent streams: each kernel's own duration):
#   tools/prof_split1.sh <tag> <config> [<config>...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; shift
OUT=gpurun_out/profs1_${TAG}
mkdir -p "$OUT"
for C in "$@"; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$C" -o run --output-format csv \
    -- python3 bench.py --config "$C" --split 1 --extras none --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/${C}_bench.json" 2> "$OUT/${C}.err" || exit 1
  find "$OUT/$C" -name '*kernel_stats.csv' -exec cp {} "$OUT/${C}_kernel_stats.csv" \;
  rm -rf "$OUT/$C"
  python3 tools/kstats.py "$OUT/${C}_kernel_stats.csv"
done
