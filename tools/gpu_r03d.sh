set -e
O=gpurun_out/r03d
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
timeout -k 10 200 python tools/plugin_profile.py 100 > $O/plugin_profile.txt 2>&1
timeout -k 10 200 python bench.py --split 1 --extras none --no-cpu-baseline > $O/bench_split1.json 2> $O/split1.err
timeout -k 10 200 python bench.py --config C4 --split 1 --extras none --no-cpu-baseline > $O/bench_c4_split1.json 2> $O/c4split1.err
