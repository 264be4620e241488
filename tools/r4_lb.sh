#!/bin/bash
# Loopback per-rank cost of the sharded path (tools/loopback_bench.py):
# G = 8, 25M reads per rank, exchange and broadcast modes, C2 and C4 tables.
# Usage: tools/r4_lb.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
T="timeout -k 10 300"
$T python3 tools/loopback_bench.py 8 25000000 1 1677721600 1 1e9 > "$out/lb_g8_exchange_c2.json" 2> "$out/lb.err" && tail -1 "$out/lb_g8_exchange_c2.json" &&
$T python3 tools/loopback_bench.py 8 25000000 1 1677721600 0 1e9 > "$out/lb_g8_broadcast_c2.json" 2>> "$out/lb.err" && tail -1 "$out/lb_g8_broadcast_c2.json" &&
$T python3 tools/loopback_bench.py 8 12500000 1 838860800 1 8e9 > "$out/lb_g8_exchange_c4.json" 2>> "$out/lb.err" && tail -1 "$out/lb_g8_exchange_c4.json" || { tail -20 "$out/lb.err"; exit 1; }
