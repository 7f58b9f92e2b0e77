set -e
O=gpurun_out/c1; mkdir -p $O
export TMPDIR=/tmp
for L in 1 2 3; do timeout -k 10 100 python bench.py --clients 1 --steps 50 --warmup 5 --lanes $L --no-cpu-baseline > $O/b_l$L.json 2>&1; done
D=/tmp/trc1; timeout -k 10 200 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --clients 1 --steps 20 --warmup 3 --no-cpu-baseline > $O/tr.json 2> $O/tr.err
python3 tools/timeline.py $D --dump 30 > $O/timeline.txt; rm -rf $D
