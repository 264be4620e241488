#!/bin/bash
# Build tools/chunk_check.cpp against khmer_amd/libkhmer_hip.so (host only).
set -euo pipefail
root="$(cd "$(dirname "$0")/.." && pwd)"
out=${1:-/tmp/chunk_check}
g++ -O2 -std=c++17 -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -o "$out" "$root/tools/chunk_check.cpp" \
    -L"$root/khmer_amd" -lkhmer_hip -Wl,-rpath,"$root/khmer_amd" -Wl,-rpath,/opt/rocm/lib
echo "built $out"
