#!/bin/bash
# End-of-round check on one MI355X: the whole -m gpu suite (timed), smoke()
# and a 20-step default bench line.  Usage: tools/final_check.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$tag
t0=$(date +%s)
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 170 --timeout-method thread \
    > gpurun_out/$tag/gpu_tests.txt 2>&1 || { echo "gpu suite failed"; tail -40 gpurun_out/$tag/gpu_tests.txt; exit 1; }
echo "suite $(( $(date +%s) - t0 )) s"; tail -2 gpurun_out/$tag/gpu_tests.txt
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/$tag/smoke.txt 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/$tag/smoke.txt; exit 1; }
tail -1 gpurun_out/$tag/smoke.txt
timeout -k 10 400 python -u bench.py --steps 20 --warmup 2 > gpurun_out/$tag/bench.json 2> gpurun_out/$tag/bench.err || { echo "bench failed"; tail -20 gpurun_out/$tag/bench.err; exit 1; }
cat gpurun_out/$tag/bench.json
