set -e
export TMPDIR=/tmp
O=gpurun_out/r2f
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for L in 1 2 3; do timeout -k 10 150 python bench.py --steps 20 --warmup 3 --lanes $L --no-cpu-baseline > $O/b_l$L.log 2>&1; done
for L in 1 2; do D=/tmp/tr$L; timeout -k 10 240 rocprofv3 --kernel-trace -d $D -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes $L --no-cpu-baseline > $O/tr$L.json 2> $O/tr$L.err; python3 tools/timeline.py $D --dump 36 > $O/timeline_l$L.txt; rm -rf $D; done
