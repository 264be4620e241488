#!/bin/bash
# Profiles the default bench workload on the GPU box (run through gpurun):
#   1. rocprofv3 --kernel-trace --stats  -> per-kernel average durations
#   2. two separate --pmc passes (FETCH_SIZE, WRITE_SIZE) -> HBM bytes
# then tools/pmc_summary.py writes profiles/<tag>_* and profiles/pmc_traffic.json.
# Usage: tools/profile_round.sh <tag> [bench args...]   (e.g. r1_v3; r5_c4 --config C4)
set -euo pipefail
tag=${1:?tag}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/prof_$tag
rm -rf "$out"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/trace" -o run --output-format csv -- \
    python3 bench.py --steps 2 --warmup 1 --cpu-reads 0 "$@" > "$out/bench.json" 2> "$out/trace.err"
for c in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --kernel-trace --pmc $c -d "$out/pmc_$c" -o run --output-format csv -- \
        python3 bench.py --steps 1 --warmup 0 --cpu-reads 0 "$@" > "$out/pmc_$c.json" 2> "$out/pmc_$c.err"
done
# summarise locally after gpurun merges gpurun_out/: python3 tools/pmc_summary.py "$out" "$tag"
