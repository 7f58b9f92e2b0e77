set -e
export TMPDIR=/tmp
O=gpurun_out/r2
mkdir -p $O
for L in 2 3; do timeout -k 10 240 rocprofv3 --kernel-trace -d $O/tr$L -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --lanes $L --no-cpu-baseline > $O/tr$L.json 2> $O/tr$L.err; python3 tools/timeline.py $O/tr$L --dump 40 > $O/timeline_l$L.txt; done
timeout -k 10 120 ./tools/scan_ablate > $O/scan_ablate.log 2>&1
timeout -k 10 120 ./tools/hbm_probe > $O/hbm_probe.log 2>&1
