set -e
O=gpurun_out/r03n
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_aggregate.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg_default.json 2>&1
for v in nox x_w4_d8 x_w4_d16 x_w3_d8; do
  COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python tools/bench_aggregate.py > $O/$v.json 2>&1
done
for f in $O/*.json; do echo $f $(grep -o '"k_aggregate_ms": [0-9.]*\|"bit_identical_to_unfused": [a-z]*' $f); done
