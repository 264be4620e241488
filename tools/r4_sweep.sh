#!/bin/bash
# Same-box C2 timing under level-1 / level-2 block and chunk knobs
# (development A/B).  Usage: tools/r4_sweep.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
run() {
    local name=$1; shift
    timeout -k 10 200 env "$@" python3 bench.py --steps 3 --warmup 1 --cpu-reads 0 --no-unprofiled > "$out/$name.json" 2> "$out/$name.err" || { echo "FAIL $name"; tail -3 "$out/$name.err"; return 1; }
    python3 -c "import json,sys; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); print('$name', round(d['ms_per_step'],1), d['check'].get('tables_match'), {k: round(v,1) for k, v in d['roofline']['kernels_ms_per_step'].items() if v > 1})"
}
run base0 KH_NONE=0 &&
run l1blk7 KH_L1F_BLK_SH=7 && run l1blk9 KH_L1F_BLK_SH=9 &&
run l2blk_lo KH_L2F_BLK_SH=5 && run l2blk_hi KH_L2F_BLK_SH=7 &&
run chunk16 KH_L1_CHUNK=16 && run chunk64 KH_L1_CHUNK=64 &&
run base1 KH_NONE=0
