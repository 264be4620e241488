#!/bin/bash
# SQ / LDS counter passes over one bench step (run through gpurun): where a
# kernel's wave cycles go.  Usage: tools/pmc_sq.sh <tag> [bench args...]
# Each pass is its own rocprofv3 run (gfx950 slot limits: 8 SQ counters).
set -euo pipefail
tag=${1:?tag}; shift
cd "$(dirname "$0")/.."
export TMPDIR=/tmp
out=gpurun_out/sq_$tag
rm -rf "$out"; mkdir -p "$out"
passes=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_WAVES"
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
)
i=0
for p in "${passes[@]}"; do
  timeout -s KILL 240 rocprofv3 --kernel-trace --pmc $p -d "$out/p$i" -o run --output-format csv -- \
      python3 bench.py --steps 1 --warmup 0 --cpu-reads 0 --no-unprofiled "$@" > "$out/p$i.json" 2> "$out/p$i.err"
  i=$((i+1))
done
