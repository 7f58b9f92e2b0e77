#!/bin/bash
# Library-variant A/B on the GPU box: tools/variant_ab.sh <tag> <command...>
# For every coala_amd/lib/variants/<name>.so: install it as the library and run <command> (one process),
# output to gpurun_out/var_<tag>/<name>.txt; prints each variant's last 3 output lines.
set -e
TAG=$1; shift
O=gpurun_out/var_${TAG}
mkdir -p $O
export TMPDIR=/tmp
for v in coala_amd/lib/variants/*.so; do
  n=$(basename $v .so)
  cp $v coala_amd/lib/libcoalac.so
  timeout -k 10 180 "$@" > $O/$n.txt 2> $O/$n.err || { tail -5 $O/$n.err; exit 1; }
  echo "== $n"; tail -3 $O/$n.txt
done
