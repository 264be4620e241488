#!/bin/bash
# Round-4 GPU check: windowed level 1 (l1f_windows) at the C3/C4/C5 geometries
# against the golden fixtures, a quick shard/schedule pass, and C4/C5/C5M
# bench lines for the level-1 window A/B (KH_L1_WIN) and the old exact path.
# Usage: tools/r4_check.sh <tag>  -> gpurun_out/r4_<tag>/
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
T="timeout -k 10"
$T 900 python3 -u -m pytest -x -v --timeout 600 --timeout-method thread tests/test_gpu_full.py \
    -k "c4_shape or c5_shape or c5m_shape or c3_shape" > "$out/full.txt" 2>&1 || { echo "full tests failed"; tail -30 "$out/full.txt"; exit 1; }
tail -3 "$out/full.txt"
$T 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_shard.py \
    -k "matches_oracle or schedules or saturated" > "$out/shard.txt" 2>&1 || { echo "shard tests failed"; tail -30 "$out/shard.txt"; exit 1; }
tail -2 "$out/shard.txt"
b() { name=$1; shift; env "$@" > /dev/null; }
for cfg in C4 C5 C5M; do
  for v in "KH_L1_WIN=1024" "KH_L1_WIN=512" "KH_L1_EXACT=1"; do
    env $v $T 300 python3 bench.py --config $cfg --steps 2 --cpu-reads 0 --no-unprofiled > "$out/${cfg}_$v.json" 2> "$out/${cfg}_$v.err" || { echo "bench $cfg $v failed"; tail -5 "$out/${cfg}_$v.err"; exit 1; }
    python3 -c "
import json,sys; d=json.loads(open('$out/${cfg}_$v.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$cfg $v', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], r['kernels_ms_per_step'])"
  done
done
