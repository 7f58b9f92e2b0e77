#!/bin/bash
# Interleaved A/B of library variants on tools/bench_aggregate.py (run through gpurun from the repo root):
#   tools/ab_aggregate.sh <tag> <rounds> <variant> [<variant> ...]   -> gpurun_out/abagg_<tag>.txt
set -e
TAG=$1; R=$2; shift 2
OUT=gpurun_out/abagg_${TAG}.txt
: > "$OUT"
for r in $(seq 1 "$R"); do
  for v in "$@"; do
    COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python3 tools/bench_aggregate.py --steps 40 > gpurun_out/abagg_last.json 2>/dev/null
    python3 - "$v" "$OUT" <<'PY'
import json, sys
d = json.loads(open("gpurun_out/abagg_last.json").read().strip().splitlines()[-1])
keep = {"ms": d["ms"], "k_aggregate_ms": d["k_aggregate_ms"], "frac": d["roofline"]["frac"], "same": d["bit_identical_to_unfused"]}
line = f"{sys.argv[1]:12s} {json.dumps(keep)}"
print(line)
open(sys.argv[2], "a").write(line + "\n")
PY
  done
done
