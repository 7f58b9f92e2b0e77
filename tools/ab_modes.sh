#!/bin/bash
# Encode-mode A/B on the GPU box: tools/ab_modes.sh <tag> — GPU fused/parity tests, then the bench
# (C3 + extras) with the default kernel sequence, the one-launch k_fused (--flags 64) and the front
# launch (--flags 128). Summary lines at the end; JSON per mode in gpurun_out/modes_<tag>/.
set -e
TAG=${1:-x}
O=gpurun_out/modes_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_parity.py tests/test_reference_fixture.py \
  -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for m in 0 64 128; do
  timeout -k 10 240 python bench.py --no-cpu-baseline --steps 10 --flags $m > $O/m$m.json 2> $O/m$m.err \
    || { tail -5 $O/m$m.err; exit 1; }
done
python - <<PY
import json
for m in (0, 64, 128):
    d = json.load(open("$O/m%d.json" % m))
    row = ["flags=%d" % m, "C3 %.0f %.3fms %s" % (d["value"], d["ms_per_step"], d["stages_ms"])]
    for k, v in d.get("configs", {}).items():
        row.append("%s %.0f %.3fms %s" % (k, v["value"], v["ms_per_step"], v["stages_ms"]))
    print(" | ".join(row))
PY
