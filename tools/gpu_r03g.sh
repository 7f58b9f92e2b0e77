set -e
O=gpurun_out/r03g
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 ./tools/store_probe2 832 1536 > $O/store_probe2.txt 2>&1
B="--extras none --no-cpu-baseline"
timeout -k 10 120 python bench.py $B > $O/c3_lds.json
COALAC_LIB=coala_amd/lib/variants/dec_reg.so timeout -k 10 120 python bench.py $B > $O/c3_reg.json
COALAC_LIB=coala_amd/lib/variants/dec_lds_dpw1.so timeout -k 10 120 python bench.py $B > $O/c3_lds_dpw1.json
COALAC_LIB=coala_amd/lib/variants/dec_lds_w8.so timeout -k 10 120 python bench.py $B > $O/c3_lds_w4.json
timeout -k 10 120 python bench.py $B --split 1 > $O/c3s1_lds.json
COALAC_LIB=coala_amd/lib/variants/dec_reg.so timeout -k 10 120 python bench.py $B --split 1 > $O/c3s1_reg.json
timeout -k 10 120 python bench.py $B --config single > $O/single_fa.json
timeout -k 10 120 python bench.py $B --config single --fill-ahead off > $O/single_nofa.json
timeout -k 10 200 python tools/plugin_profile.py 100 > $O/plugin_profile.txt 2>&1
timeout -k 10 200 python tools/host_rate.py --clients 1 > $O/host_rate.jsonl 2> $O/host_rate.err
timeout -k 10 120 python tools/bench_aggregate.py > $O/aggregate.json 2>&1
