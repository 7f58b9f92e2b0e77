# GPU suite + the bench (default: all extras): tools/gpu_suite_bench.sh <tag> [<bench args>...]
set -o pipefail
export TMPDIR=/tmp
O=gpurun_out/$1
shift
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline "$@" > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]); print(len(json.dumps(d))); print(json.dumps(d['configs_summary']))"
