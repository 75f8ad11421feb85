#!/bin/bash
# ASan + UBSan build of the host runtime: build/asan/_C_host_asan.so.  Load it with
# LD_PRELOAD=$(gcc -print-file-name=libasan.so) (see tests/test_sanitize_host.py).
set -eu
R=$(cd "$(dirname "$0")/../.." && pwd)
out=$R/build/asan
mkdir -p "$out"
read -r TINC TLIB ABI PYINC < <(python3 -c "
import os, sysconfig, torch
d = os.path.dirname(torch.__file__)
print(f'{d}/include', f'{d}/lib', int(torch._C._GLIBCXX_USE_CXX11_ABI), sysconfig.get_paths()['include'])")
FLAGS="-O1 -g -std=c++17 -fPIC -fno-omit-frame-pointer -fsanitize=address,undefined -fno-sanitize-recover=undefined -D_GLIBCXX_USE_CXX11_ABI=$ABI -DTORCH_EXTENSION_NAME=_C_host_asan -DTORCH_API_INCLUDE_EXTENSION_H -I$TINC -I$TINC/torch/csrc/api/include -I$PYINC"
g++ $FLAGS -c "$R/multigrad_amd/csrc/runtime.cpp" -o "$out/runtime.o"
g++ $FLAGS -c "$R/tools/sanitize/host_bindings.cpp" -o "$out/host_bindings.o"
g++ -shared -fsanitize=address,undefined -o "$out/_C_host_asan.so" "$out/runtime.o" "$out/host_bindings.o" \
  -L"$TLIB" -lc10 -ltorch -ltorch_cpu -ltorch_python -Wl,-rpath,"$TLIB"
echo "$out/_C_host_asan.so"
