set -e
O=gpurun_out/r03i
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_default.json 2>&1
for v in agg_s4 agg_s4d16 agg_s4d4 agg_s2w2; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/$v.json 2>&1
done
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
