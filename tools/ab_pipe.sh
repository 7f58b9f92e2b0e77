#!/bin/bash
# Pipeline A/B on the GPU box: tools/ab_pipe.sh <tag> — pipeline parity tests, then the headline bench
# (C3 share) as free-running SplitPipeline sub-batches vs LanePipeline lanes (streaming kernels back to back
# on one stream: one read phase, then one write phase), and the single update as lanes. Summary at the end;
# JSON per run in gpurun_out/pipe_<tag>/.
set -e
TAG=${1:-x}
O=gpurun_out/pipe_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q --timeout 120 --timeout-method thread \
  > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # name, bench args...
  local n=$1; shift
  timeout -k 10 180 python bench.py --no-cpu-baseline --extras none --steps 40 "$@" > $O/$n.json 2> $O/$n.err \
    || { tail -5 $O/$n.err; exit 1; }
}
run split2 --split 2
run lane2 --pipe lane --split 2
run lane3 --pipe lane --split 3
run lane4 --pipe lane --split 4
run split2b --split 2
run lane2b --pipe lane --split 2
run c4split2 --config C4 --split 2 --steps 10
run c4lane2 --config C4 --pipe lane --split 2 --steps 10
run c4lane3 --config C4 --pipe lane --split 3 --steps 10
run single --config single --steps 100
run single_lane2 --config single --pipe lane --split 2 --steps 100
run single_lane3 --config single --pipe lane --split 3 --steps 100
python - <<PY
import json, glob, os
for f in sorted(glob.glob("$O/*.json")):
    d = json.load(open(f))
    print("%-14s %8.1f GB/s  %.4f ms  step_roof %.3f  %s" % (os.path.basename(f)[:-5], d["value"], d["ms_per_step"],
          d.get("step_roofline", {}).get("frac", 0), d.get("stages_ms")))
PY
