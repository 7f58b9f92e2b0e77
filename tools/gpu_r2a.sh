set -e
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
for L in 1 2 3 4; do timeout -k 10 150 python bench.py --steps 20 --warmup 3 --lanes $L --no-cpu-baseline > $O/b_l$L.log 2>&1; done
timeout -k 10 150 python bench.py --steps 20 --warmup 3 --lanes 2 --clients 1 --no-cpu-baseline > $O/b_c1_l2.log 2>&1
for L in 1 2; do timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr$L -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes $L --no-cpu-baseline > $O/tr$L.json 2> $O/tr$L.err; python3 tools/timeline.py $O/tr$L > $O/timeline_l$L.json; done
timeout -k 10 120 ./tools/scan_ablate > $O/scan_ablate.log 2>&1
timeout -k 10 120 ./tools/hbm_probe > $O/hbm_probe.log 2>&1
