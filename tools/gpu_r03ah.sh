#!/bin/bash
# k_sample: the segment record from lsegs (same load round as the segment index) instead of segs[large_list[li]].
set -e
O=gpurun_out/r03ah
mkdir -p $O
export TMPDIR=/tmp
L=coala_amd/lib/variants
COALAC_LIB=$L/samp1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_mixed.py -x -q \
  --timeout 120 --timeout-method thread > $O/pytest.log 2>&1 || { tail -40 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
B="--extras none --no-cpu-baseline --steps 300 --warmup 20"
for i in 1 2 3 4; do
  timeout -k 10 120 python bench.py $B --config single > $O/single_def_$i.json 2>>$O/err.log
  COALAC_LIB=$L/samp1.so timeout -k 10 120 python bench.py $B --config single > $O/single_samp1_$i.json 2>>$O/err.log
  timeout -k 10 120 python bench.py $B --config C5 > $O/c5_def_$i.json 2>>$O/err.log
  COALAC_LIB=$L/samp1.so timeout -k 10 120 python bench.py $B --config C5 > $O/c5_samp1_$i.json 2>>$O/err.log
done
for i in 1 2; do
  timeout -k 10 120 python bench.py --extras none --no-cpu-baseline > $O/c3_def_$i.json 2>>$O/err.log
  COALAC_LIB=$L/samp1.so timeout -k 10 120 python bench.py --extras none --no-cpu-baseline > $O/c3_samp1_$i.json 2>>$O/err.log
done
for f in $O/*.json; do echo $(basename $f) $(python -c "import json; d=json.load(open('$f')); print(d['value'], d['ms_per_step'])"); done
