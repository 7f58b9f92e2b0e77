# rocprof kernel stats of configs under an env toggle: tools/prof_env.sh <tag> "<ENV=..>" <config> [<config>...]
set -o pipefail
export TMPDIR=/tmp
TAG=$1; E=$2; shift 2
OUT=gpurun_out/profc_${TAG}
mkdir -p "$OUT"
for C in "$@"; do
  env $E timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$OUT/$C" -o run --output-format csv \
    -- python3 bench.py --config "$C" --extras none --no-cpu-baseline --steps 20 --warmup 3 > "$OUT/${C}_bench.json" 2> "$OUT/${C}.err" || exit 1
  find "$OUT/$C" -name '*kernel_stats.csv' -exec cp {} "$OUT/${C}_kernel_stats.csv" \;
  rm -rf "$OUT/$C"
  grep -v "at::\|__amd" "$OUT/${C}_kernel_stats.csv" | cut -d, -f1,3,4 | cut -c1-150
done
