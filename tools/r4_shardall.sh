#!/bin/bash
# The whole sharded suite (loopback, multi-process, RCCL at world 1) with
# progress on stderr.  Usage: tools/r4_shardall.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
timeout -k 10 1100 python3 -u -m pytest -x -v -s --timeout 500 --timeout-method thread \
    tests/test_gpu_shard.py tests/test_gpu_shard_mp.py > "$out/shard_all.txt" 2>&1
rc=$?
grep -E "FAILED|ERROR|passed|failed" "$out/shard_all.txt" | tail -10
exit $rc
