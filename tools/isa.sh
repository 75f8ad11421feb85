#!/bin/bash
# Device assembly of one csrc/*.hip file for gfx950 (extra -D flags pass through), plus a
# per-kernel instruction census of the main loop: bash tools/isa.sh smf [-DMG_X=1 ...]
set -eu
R=$(cd "$(dirname "$0")/.." && pwd)
src=$1; shift
out=${ISA_OUT:-/tmp/isa}/$src.s
mkdir -p "$(dirname "$out")"
inc=$(python3 -c "import torch,os;d=os.path.dirname(torch.__file__);print(f'-I{d}/include -I{d}/include/torch/csrc/api/include')")
pyinc=$(python3 -c "import sysconfig;print(sysconfig.get_paths()['include'])")
/opt/rocm/bin/hipcc --offload-arch=gfx950 --cuda-device-only -S -O3 -std=c++17 -ffp-contract=fast \
  -D__HIP_PLATFORM_AMD__=1 -DUSE_ROCM=1 -DTORCH_EXTENSION_NAME=_C -DTORCH_API_INCLUDE_EXTENSION_H \
  -I"$R/multigrad_amd/csrc" -I"$pyinc" $inc "$@" "$R/multigrad_amd/csrc/$src.hip" -o "$out"
echo "$out"
