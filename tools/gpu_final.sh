#!/bin/bash
# Round-end evidence on the GPU box: GPU tests, smoke(), the default bench line (all extras, CPU baseline),
# then tools/profile_round.sh <tag> (kernel stats, PMC traffic, union timeline). tools/gpu_final.sh <tag>
set -e
TAG=${1:-r02}
O=gpurun_out/final_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
echo "bench done"
bash tools/profile_round.sh $TAG > $O/profile.log 2>&1 || { tail -20 $O/profile.log; exit 1; }
echo "profile done"
