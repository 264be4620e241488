#!/bin/bash
# Tagging path (consume_seqfile_and_tag) after the bitmap / host-hash / flat
# tag-set rewrite: parity tests, then the end-to-end line.  Usage: tools/r4_tag.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
    tests/test_gpu_robust.py tests/test_gpu_scripts.py -k "tag or load_graph or concurrent" > "$out/tag_tests.txt" 2>&1 || { tail -30 "$out/tag_tests.txt"; exit 1; }
grep -E "PASSED|FAILED|passed|failed" "$out/tag_tests.txt" | tail -20
timeout -k 10 300 python3 tools/bench_e2e.py --tag --reads 5000000 --cpu-reads 100000 > "$out/e2e_tag.json" 2> "$out/e2e_tag.err" || { tail -5 "$out/e2e_tag.err"; exit 1; }
tail -1 "$out/e2e_tag.json"
