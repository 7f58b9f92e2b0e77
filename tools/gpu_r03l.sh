set -e
O=gpurun_out/r03l
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_aggregate.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_default.json 2>&1
for v in agg_d4 agg_d16; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/$v.json 2>&1
done
tail -n 3 $O/*.json
