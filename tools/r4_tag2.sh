#!/bin/bash
# Tagging path after the prefetched tag inserts, then C4 in loopback exchange.
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
bash tools/r4_tag.sh "$tag" &&
timeout -k 10 300 python3 tools/loopback_bench.py 8 12500000 1 838860800 1 8e9 > "$out/lb_g8_exchange_c4.json" 2> "$out/lb_c4.err" && tail -1 "$out/lb_g8_exchange_c4.json"
