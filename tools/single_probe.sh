#!/bin/bash
# One library variant's single-update numbers (run from tools/variant_ab.sh, which installs the variant):
# two 'single' bench lines, then a rocprofv3 kernel-stats pass whose codec rows are printed.
#   tools/variant_ab.sh <tag> bash tools/single_probe.sh <outdir-prefix>
set -e
P=${1:-gpurun_out/sp}
N=$(md5sum coala_amd/lib/libcoalac.so | cut -c1-8)
O=${P}_$N
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2; do
  timeout -k 10 120 python bench.py --config single --extras none --no-cpu-baseline --steps 300 --warmup 20 ${SP_ARGS} \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('single', d['value'], d['ms_per_step'], d['step_roofline']['frac'])"
done
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv \
  -- python3 bench.py --config single --extras none --no-cpu-baseline --steps 40 --warmup 5 ${SP_ARGS} > $O/b.json 2> $O/prof.err
f=$(find $O/prof -name '*kernel_stats.csv' | head -1)
python3 tools/filter_stats.py $f $O/stats.csv
rm -rf $O/prof
cut -d, -f1-4 $O/stats.csv | sed 's/"//g' | awk -F, 'NR>1 && $1 !~ /other/ {printf "  %-40s %8.2f us\n", $1","$2, $4/1000}'
