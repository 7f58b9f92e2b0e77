#!/bin/bash
# A/B of the one-launch encode on the GPU box: tools/sweep_fused.sh <tag> "<delays>" [extra bench args]
# Runs the fused-path tests first, then the bench (C3 headline + extras) per COALAC_FUSED_DELAY and once
# with the multi-launch encode (--flags 16). One line per run in gpurun_out/sweep_<tag>/runs.jsonl.
set -e
TAG=${1:-x}
DELAYS=${2:-"1024"}
shift 2 || true
O=gpurun_out/sweep_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_reference_fixture.py -x -q --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for d in $DELAYS; do
  COALAC_FUSED_DELAY=$d timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 "$@" > $O/d$d.json 2> $O/d$d.err \
    || { tail -5 $O/d$d.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$O/d$d.json')); d['delay']=$d; print(json.dumps(d))" >> $O/runs.jsonl
done
timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --flags 16 "$@" > $O/multi.json 2> $O/multi.err \
  || { tail -5 $O/multi.err; exit 1; }
python -c "import json; d=json.load(open('$O/multi.json')); d['delay']='multi'; print(json.dumps(d))" >> $O/runs.jsonl
python - <<PY
import json
for l in open("$O/runs.jsonl"):
    d = json.loads(l)
    row = [str(d["delay"]), "C3 %.0f %.3fms %s" % (d["value"], d["ms_per_step"], d["stages_ms"])]
    for k, v in d.get("configs", {}).items():
        row.append("%s %.0f %.3fms %s" % (k, v["value"], v["ms_per_step"], v["stages_ms"]))
    print(" | ".join(row))
PY
