set -e
O=gpurun_out/r03r
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
B="--extras none --no-cpu-baseline"
for i in 1 2 3; do
timeout -k 10 120 python bench.py $B > $O/defer_$i.json
COALAC_LIB=coala_amd/lib/variants/nodefer.so timeout -k 10 120 python bench.py $B > $O/nodefer_$i.json
done
for f in $O/*.json; do echo $f $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $f); done
