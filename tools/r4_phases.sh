#!/bin/bash
# Phase stamps (-DKH_PHASES build in abx/libphases.so) of the C2 and C4
# workloads (tools/phase_probe.py).  Usage: tools/r4_phases.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
KHMER_AMD_LIB=abx/libphases.so timeout -k 10 300 python3 tools/phase_probe.py 50000000 1e9 > "$out/phases_c2.txt" 2>&1 &&
KHMER_AMD_LIB=abx/libphases.so timeout -k 10 300 python3 tools/phase_probe.py 50000000 8e9 > "$out/phases_c4.txt" 2>&1
rc=$?
tail -12 "$out/phases_c2.txt" "$out/phases_c4.txt"
exit $rc
