set -e
O=gpurun_out/r03k
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_aggregate.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2; do
timeout -k 10 120 python bench.py $B > $O/c3_lean_$i.json
COALAC_LIB=coala_amd/lib/variants/scan_nolean.so timeout -k 10 120 python bench.py $B > $O/c3_nolean_$i.json
done
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_default.json 2>&1
for v in agg_s4d4w4 agg_s4d8w4; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/$v.json 2>&1
done
