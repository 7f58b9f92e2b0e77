#!/bin/bash
# single update: decode background beside the encode (fill-ahead after k_scan / at the start) with a full-grid
# or a bounded-grid k_fill (FILL_BLOCKS variants), against the default k_fillscatter sequence.
set -e
O=gpurun_out/r03u
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_pipeline.py -x -q -k fill_ahead --timeout 120 \
  --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--config single --extras none --no-cpu-baseline --steps 300 --warmup 20"
for i in 1 2; do
  for fa in off on start; do
    timeout -k 10 120 python bench.py $B --fill-ahead $fa > $O/def_${fa}_$i.json 2>>$O/err.log
  done
  for v in fill256 fill512 fill1024; do
    for fa in on start; do
      COALAC_LIB=coala_amd/lib/variants/$v.so timeout -k 10 120 python bench.py $B --fill-ahead $fa > $O/${v}_${fa}_$i.json 2>>$O/err.log
    done
  done
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json,sys; d=json.load(open('$f')); print(d['value'], d['ms_per_step'], d['config'].get('graph'), d['config'].get('fill_ahead'))"); done
