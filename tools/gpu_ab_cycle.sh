#!/bin/bash
# One build -> measure cycle on the GPU box: GPU tests on the in-tree library, then every library variant
# under coala_amd/lib/variants: single-update kernel stats (tools/single_probe.sh) and two C3 bench lines.
#   tools/gpu_ab_cycle.sh <tag> [pytest selection]
set -e
TAG=${1:-ab}
SEL=${2:-tests}
O=gpurun_out/cyc_${TAG}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest $SEL -m gpu -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 \
  || { tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
cp coala_amd/lib/libcoalac.so $O/in_tree.so.bak
for v in coala_amd/lib/variants/*.so; do
  n=$(basename $v .so)
  cp $v coala_amd/lib/libcoalac.so
  bash tools/single_probe.sh $O/sp_$n > $O/$n.txt 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  for i in 1 2; do
    timeout -k 10 120 python bench.py --no-cpu-baseline --extras none \
      | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('C3', d['value'], d['ms_per_step'])" >> $O/$n.txt
  done
  echo "== $n"; grep -E "^single|^C3" $O/$n.txt
done
cp $O/in_tree.so.bak coala_amd/lib/libcoalac.so && rm $O/in_tree.so.bak
# optional: single-update lines of the in-tree library with extra bench flags, e.g. EXTRA_FLAGS="0 64 128"
for f in ${EXTRA_FLAGS}; do
  timeout -k 10 120 python bench.py --config single --extras none --no-cpu-baseline --steps 300 --warmup 20 --flags $f \
    | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('single flags=$f', d['value'], d['ms_per_step'])"
done
