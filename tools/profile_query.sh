#!/bin/bash
# Profiles the C5 get_median_count query line (bench.py --config C5 --query)
# on the GPU box: kernel trace + separate FETCH_SIZE / WRITE_SIZE passes.
# Usage: tools/profile_query.sh <tag>  -> gpurun_out/profq_<tag>/
# Summarise locally: python3 tools/pmc_summary.py gpurun_out/profq_<tag> <tag>_query
set -euo pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/profq_$tag
rm -rf "$out"
mkdir -p "$out"
args="--config C5 --query --steps 1 --warmup 0 --cpu-reads 0 --no-unprofiled"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
    python3 bench.py $args > "$out/bench.json" 2> "$out/trace.err"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$out/pmc_$c" -o run --output-format csv -- \
        python3 bench.py $args > "$out/pmc_$c.json" 2> "$out/pmc_$c.err"
done
