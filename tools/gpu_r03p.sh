set -e
O=gpurun_out/r03p
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_aggregate.py tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--extras none --no-cpu-baseline --mode delta"
for i in 1 2; do
timeout -k 10 120 python bench.py $B > $O/delta_new_$i.json
COALAC_LIB=coala_amd/lib/variants/dec_old.so timeout -k 10 120 python bench.py $B > $O/delta_old_$i.json
done
timeout -k 10 120 python tools/bench_aggregate.py > $O/agg.json 2>&1
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"k_aggregate_ms": [0-9.]*\|"bit_identical_to_unfused": [a-z]*' $f); done
