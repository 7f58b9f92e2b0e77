#!/bin/bash
# Full round check on the GPU box (run through gpurun from the repo root): tools/gpu_full.sh <tag>
# GPU tests, smoke(), the default bench line, then tools/profile_round.sh <tag>.
set -e
TAG=${1:-r01}
O=gpurun_out/full_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
timeout -k 10 200 python bench.py > $O/bench.json 2> $O/bench.err
bash tools/profile_round.sh $TAG
