#!/bin/bash
# Batch small-segment limit 1024 as the default: GPU suite, smoke, default bench line, and C2 / C3 / C4 against
# the old 4096 (COALAC_SMALL_MAX=4096) interleaved.
set -e
O=gpurun_out/r03al
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
print("C3", d["value"], d["ms_per_step"], d["step_roofline"]["frac"], d["roofline"]["kernel"], d["roofline"]["frac"], d["roofline"]["traffic"])
for k, v in d["configs"].items():
    print(k, v["value"], v.get("ms_per_step", v.get("ms_per_client")), v["step_roofline"]["frac"])
print("cpu", d["cpu_baseline"]["value"], d["cpu_baseline"]["cores"])
PY
B="--extras none --no-cpu-baseline"
for i in 1 2; do
  for c in C2 C3 C4; do
    timeout -k 10 120 python bench.py $B --config $c > $O/${c}_new_$i.json 2>>$O/err.log
    COALAC_SMALL_MAX=4096 timeout -k 10 120 python bench.py $B --config $c > $O/${c}_old_$i.json 2>>$O/err.log
  done
done
for f in $O/C*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['stages_ms'])"); done
