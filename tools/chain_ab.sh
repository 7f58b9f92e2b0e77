#!/bin/bash
# Kernel-variant A/B of the latency chain on the GPU box: tools/chain_ab.sh <tag> [probe args]
# For every coala_amd/lib/variants/<name>.so (built here with different -D knobs): install it as the
# library, run tools/chain_probe.py --stages under rocprofv3 --kernel-trace --stats, keep the kernel stats.
# Prints one line per variant: the round trip and each kernel's mean duration (us).
set -e
TAG=${1:-x}; shift || true
O=gpurun_out/chain_${TAG}
mkdir -p $O
export TMPDIR=/tmp
for v in coala_amd/lib/variants/*.so; do
  n=$(basename $v .so)
  cp $v coala_amd/lib/libcoalac.so
  timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$n -o run --output-format csv \
    -- python3 tools/chain_probe.py --stages "$@" > $O/$n.txt 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  find $O/$n -name '*kernel_stats.csv' -exec cp {} $O/$n.stats.csv \;
  rm -rf $O/$n
  if [ -n "$BENCH" ]; then  # also the headline bench (C3 share) and the single extra, no profiler
    timeout -k 10 180 python3 bench.py --no-cpu-baseline --extras single --steps 40 > $O/$n.bench.json 2> $O/$n.bench.err \
      || { tail -5 $O/$n.bench.err; exit 1; }
  fi
done
python3 - <<PY
import csv, glob, os, re
for f in sorted(glob.glob("$O/*.stats.csv")):
    n = os.path.basename(f)[:-10]
    rows = {}
    for r in csv.DictReader(open(f)):
        m = re.search(r"\b(k_\w+)", r["Name"])
        if m:
            rows[m.group(1)] = float(r["AverageNs"]) / 1e3
    rt = open("$O/%s.txt" % n).read().strip()
    print(n, "|", rt, "|", " ".join("%s=%.1f" % kv for kv in sorted(rows.items())))
    if os.path.exists("$O/%s.bench.json" % n):
        import json
        d = json.load(open("$O/%s.bench.json" % n))
        s1 = d["configs"]["single"]
        print("   C3 %.1f GB/s %.4f ms | single %.1f GB/s %.4f ms" % (d["value"], d["ms_per_step"], s1["value"], s1["ms_per_step"]))
PY
