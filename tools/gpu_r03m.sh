set -e
O=gpurun_out/r03m
mkdir -p $O
export TMPDIR=/tmp
for v in agg_p1 agg_p2 agg_s4 agg_d8 agg_d16; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/$v.json 2>&1
done
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_default.json 2>&1
grep -h -o '"k_aggregate_ms": [0-9.]*\|"bit_identical_to_unfused": [a-z]*' $O/*.json
