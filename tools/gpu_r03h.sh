set -e
O=gpurun_out/r03h
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
B="--extras none --no-cpu-baseline"
timeout -k 10 120 python bench.py $B --split 3 > $O/c3_split3.json
timeout -k 10 120 python bench.py $B --split 4 > $O/c3_split4.json
timeout -k 10 120 python bench.py $B --config C4 --split 1 > $O/c4_split1.json
timeout -k 10 120 python bench.py $B --config C2 --split 2 > $O/c2_split2.json
bash tools/profile_round.sh r03 > $O/profile.log 2>&1
