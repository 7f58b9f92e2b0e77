set -e
O=gpurun_out/r03f
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 200 python tools/plugin_profile.py 100 > $O/plugin_profile.txt 2>&1
timeout -k 10 200 python tools/host_rate.py --clients 1 > $O/host_rate.jsonl 2> $O/host_rate.err
timeout -k 10 120 ./tools/store_probe2 832 1536 > $O/store_probe2.txt 2>&1
