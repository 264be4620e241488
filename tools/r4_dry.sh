#!/bin/bash
# Multi-rank dry run of bench.py on one GPU (host transport instead of RCCL):
# BASELINE C4 (4 x 8e9) over 2 ranks, exchange mode, 400K reads (strong): the
# c4_400k_x2 fixture holds that pass order, so the line's check is exact.
# Usage: tools/r4_dry.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
KH_BENCH_DEVICE=0 timeout -k 10 900 python3 bench.py --gpus 2 --config C4 --strong --reads 400000 \
    --steps 1 --warmup 1 --cpu-reads 0 --no-unprofiled > "$out/dry_c4_g2_exchange.json" 2> "$out/dry.err" || { tail -20 "$out/dry.err"; exit 1; }
tail -1 "$out/dry_c4_g2_exchange.json"
