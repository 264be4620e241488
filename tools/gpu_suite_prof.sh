#!/bin/bash
# One gpurun call: the whole -m gpu suite, then the default C2 bench profile
# (tools/profile_round.sh).  Usage: tools/gpu_suite_prof.sh <tag> [bench args]
set -o pipefail
tag=${1:?tag}; shift
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$tag
t0=$(date +%s)
timeout -k 10 840 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread \
    > gpurun_out/$tag/gpu_tests.txt 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/$tag/gpu_tests.txt; exit 1; }
echo "suite $(( $(date +%s) - t0 )) s"
tail -3 gpurun_out/$tag/gpu_tests.txt
tools/profile_round.sh "$tag" "$@" || { echo "profile failed"; exit 1; }
cat gpurun_out/prof_$tag/bench.json
