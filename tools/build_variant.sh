#!/bin/bash
# Build an A/B variant of the codec library with extra -D flags: tools/build_variant.sh <name> -DFOO=1 ...
# -> coala_amd/lib/variants/<name>.so (load it with COALAC_LIB=<path>).
set -e
NAME=$1; shift
mkdir -p coala_amd/lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 "$@" \
  -o coala_amd/lib/variants/$NAME.so coala_amd/csrc/coalac.hip
