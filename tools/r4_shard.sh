#!/bin/bash
# Round-4 GPU check of the sharded paths: Murmur groups, the sharded query,
# schedules, exact exchange-mode fixtures at c2_full / genomic_c2 / c4_shape.
# Usage: tools/r4_shard.sh <tag> [pytest -k expression]
set -u
tag=${1:?tag}
expr=${2:-"query or c5m or schedules or full_c2 or genomic or c4_shape"}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
timeout -k 10 1000 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_shard.py \
    -k "$expr" > "$out/shard.txt" 2>&1
rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" "$out/shard.txt" | tail -60
exit $rc
