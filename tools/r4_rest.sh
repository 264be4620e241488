#!/bin/bash
# Round-4 GPU tests not covered by r4_shard b: C4 groups, c5m_genomic groups,
# the 1-rank RCCL group, multi-process Murmur/query groups, C1's command and
# the genomic nibble fixtures.  Usage: tools/r4_rest.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
T="timeout -k 10"
run() {
  name=$1; shift
  $T "$@" > "$out/$name.txt" 2>&1
  rc=$?
  grep -E "PASSED|FAILED|ERROR|passed|failed" "$out/$name.txt" | tail -40
  return $rc
}
true &&
run c4 900 python3 -u -m pytest -x -v -s --timeout 400 --timeout-method thread tests/test_gpu_shard.py -k "c4_shape or c5m_genomic" &&
run mp 400 python3 -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gpu_shard_mp.py &&
run misc 500 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_scripts.py tests/test_gpu_full.py -k "c1_exact or genomic"
