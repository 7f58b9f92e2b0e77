#!/bin/bash
# New decode defaults (8-row passes, one unit per wave): full GPU suite, smoke, the default bench line; then
# whole-unit passes with 64 / 128-thread blocks and 128-thread 8-row blocks against it.
set -e
O=gpurun_out/r03z
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python bench.py > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python - $O/bench.json <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print("C3", d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"])
for k, v in d["configs"].items():
    print(k, v["value"], v.get("ms_per_step", v.get("ms_per_client")), v["step_roofline"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
B="--extras none --no-cpu-baseline"
L=coala_amd/lib/variants
for v in dq16n64 dq16n128; do
  COALAC_LIB=$L/$v.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_pipeline.py -x -q \
    --timeout 120 --timeout-method thread > $O/pytest_$v.log 2>&1 || { tail -40 $O/pytest_$v.log; exit 1; }
  echo $v; tail -1 $O/pytest_$v.log
done
for i in 1 2; do
  timeout -k 10 120 python bench.py $B > $O/c3_def_$i.json 2>>$O/err.log
  for v in dq16n64 dq16n128 n128; do
    COALAC_LIB=$L/$v.so timeout -k 10 120 python bench.py $B > $O/c3_${v}_$i.json 2>>$O/err.log
  done
done
for f in $O/c3_*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['stages_ms'])"); done
