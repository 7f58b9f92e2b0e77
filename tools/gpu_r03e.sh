set -e
O=gpurun_out/r03e
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 200 python tools/plugin_profile.py 100 > $O/plugin_profile.txt 2>&1
timeout -k 10 200 python tools/host_rate.py > $O/host_rate.jsonl 2> $O/host_rate.err
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
