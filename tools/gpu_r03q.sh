set -e
O=gpurun_out/r03q
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1 || true
grep -o "SQ_[A-Z0-9_]*" $O/counters.txt | sort -u > $O/sq_counters.txt || true
wc -l $O/sq_counters.txt
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS -d $O/p1 -o run --output-format csv -- python tools/bench_aggregate.py --steps 5 --warmup 1 > $O/p1.log 2>&1
python tools/pmc_kernel.py $O/p1 k_aggregate > $O/p1.json
cat $O/p1.json
