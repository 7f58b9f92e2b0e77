#!/bin/bash
# One GPU check on the box (through gpurun, from the repo root): tools/gpu_check.sh <tag> [pytest-args]
# GPU tests (one process), then the default bench line. Each step under its own time limit; stop at the
# first failure.
set -e
TAG=${1:-r02}
shift || true
O=gpurun_out/check_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread "$@" > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
cat $O/bench.json
