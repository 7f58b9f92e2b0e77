#!/bin/bash
# Interleaved A/B of library variants on one bench config (run through gpurun from the repo root):
#   tools/ab_variants.sh <tag> <config> <rounds> <variant> [<variant> ...]   (variants: coala_amd/lib/variants/<v>.so)
# One line per run: variant, ms_per_step, value, stages_ms -> gpurun_out/ab_<tag>.txt
set -e
TAG=$1; CFG=$2; R=$3; shift 3
OUT=gpurun_out/ab_${TAG}.txt
: > "$OUT"
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 180 python3 bench.py --config "$CFG" --extras none \
      --no-cpu-baseline --steps 60 --warmup 5 > gpurun_out/ab_${TAG}_last.json 2>/dev/null
    python3 - "$v" "$OUT" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/ab_" + sys.argv[2].split("ab_")[1].replace(".txt", "") + "_last.json").read().strip().splitlines()[-1])
line = f"{sys.argv[1]:16s} ms={d['ms_per_step']:.4f} value={d['value']:.1f} stages={d['stages_ms']} copy={d.get('box')}"
print(line)
open(sys.argv[2], "a").write(line + "\n")
PY
  done
done
