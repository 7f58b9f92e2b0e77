set -e
export TMPDIR=/tmp
O=gpurun_out/r2d
mkdir -p $O
timeout -k 10 420 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for L in 1 2 3 4; do timeout -k 10 150 python bench.py --steps 20 --warmup 3 --lanes $L --no-cpu-baseline > $O/b_l$L.log 2>&1; done
for L in 2 3; do timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr$L -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes $L --no-cpu-baseline > $O/tr$L.json 2> $O/tr$L.err; python3 tools/timeline.py $O/tr$L --dump 36 > $O/timeline_l$L.txt; done
