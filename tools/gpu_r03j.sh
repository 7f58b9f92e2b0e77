set -e
O=gpurun_out/r03j
mkdir -p $O
export TMPDIR=/tmp
COALA_BENCH_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 > $O/bench_gpus2_gloo.json 2> $O/bench_gpus2_gloo.err || { tail -30 $O/bench_gpus2_gloo.err; exit 1; }
timeout -k 10 300 python bench.py --extras plugin --no-cpu-baseline > $O/bench_plugin.json 2> $O/bench_plugin.err
