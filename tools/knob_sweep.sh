#!/bin/bash
# Same-box timing of the default C2 bench under a few engine knobs
# (development A/B; each line is one bench.py run, no CPU baseline).
# Usage (through gpurun): bash tools/knob_sweep.sh <outdir>
set -euo pipefail
cd "$(dirname "$0")/.."
out=${1:-gpurun_out/sweep}
mkdir -p "$out"
run() {  # run <name> [ENV=VAL ...]
    local name=$1; shift
    timeout -k 10 120 env "$@" python3 bench.py --steps 3 --warmup 1 --cpu-reads 0 > "$out/$name.json" 2> "$out/$name.err"
    python3 -c "import json,sys; d=json.load(open('$out/$name.json')); print('$name', round(d['ms_per_step'],1), {k: round(v,1) for k, v in d['roofline']['kernels_ms_per_step'].items() if v > 1})"
}
run base0 KH_NONE=0
run s0_13 KH_S0=13
run s2_9 KH_S2=9
run base1 KH_NONE=0
