#!/bin/bash
# Whole GPU suite, smoke, then the default bench line (the driver's BENCH
# command).  Usage: tools/r4_final.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
timeout -k 10 1500 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu > "$out/gpu_tests.txt" 2>&1 || { grep -E "FAILED|ERROR|Error" "$out/gpu_tests.txt" | head -20; tail -5 "$out/gpu_tests.txt"; exit 1; }
tail -1 "$out/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { tail -20 "$out/smoke.txt"; exit 1; }
tail -2 "$out/smoke.txt"
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -10 "$out/bench.err"; exit 1; }
tail -1 "$out/bench.json"
