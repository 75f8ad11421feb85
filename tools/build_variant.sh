#!/bin/bash
# Build an A/B variant of the extension: bash tools/build_variant.sh NAME -DFLAG=V ...
# -> variants/NAME/_C.so (compared against the in-tree build by tools/ab_variants.sh)
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
name=$1; shift
D=${VARIANT_DIR:-$R/variants}
mkdir -p "$D/$name"
MULTIGRAD_HIPCC_FLAGS="$*" MULTIGRAD_OBJ_DIR="$R/build/variants/$name" \
  MULTIGRAD_TARGET="$D/$name/_C.so" python -m multigrad_amd.ops.build
