#!/bin/bash
# Build an A/B variant of the codec library: tools/build_variant.sh <name> [-DKNOB=VALUE ...]
# -> coala_amd/lib/variants/<name>.so (load it with COALAC_LIB=<path>; tools/ab_variants.sh interleaves variants).
# The product build's tuning values are constants (`constexpr <type> KNOB = value;` in coalac.hip, each with the
# measurements that chose it): a -D of such a name rewrites that constant in a temporary copy of the source; any
# other -D (or flag) goes to hipcc as is.
set -e
NAME=$1; shift
SRC=coala_amd/csrc/coalac.hip
TMP=coala_amd/csrc/_variant_${NAME}.hip
trap 'rm -f "$TMP"' EXIT
cp "$SRC" "$TMP"
FLAGS=()
for a in "$@"; do
  if [[ $a =~ ^-D([A-Za-z_0-9]+)=(.*)$ ]] && grep -qE "^constexpr (int|uint32_t|double) ${BASH_REMATCH[1]} = " "$TMP"; then
    sed -i -E "s/^(constexpr (int|uint32_t|double) ${BASH_REMATCH[1]} = )[^;]*;/\1${BASH_REMATCH[2]};/" "$TMP"
  else
    FLAGS+=("$a")
  fi
done
mkdir -p coala_amd/lib/variants
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -shared -ffp-contract=off --offload-arch=gfx950 "${FLAGS[@]}" \
  -o coala_amd/lib/variants/$NAME.so "$TMP"
