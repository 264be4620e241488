#!/bin/bash
# A/B of the register-direct level 1 (KH_L1R) on the C2 bench, with the
# c2_full parity check of the bench line itself; then the schedule tests
# under each mode.  Usage: tools/r4_l1r.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
for m in 0 1 2; do
  KH_L1R=$m timeout -k 10 300 python3 bench.py --steps 3 --cpu-reads 0 --no-unprofiled > "$out/c2_l1r$m.json" 2> "$out/c2_l1r$m.err" || { echo "bench l1r=$m failed"; tail -5 "$out/c2_l1r$m.err"; exit 1; }
  python3 -c "
import json; d=json.loads(open('$out/c2_l1r$m.json').read().strip().splitlines()[-1]); r=d['roofline']
print('l1r=$m', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], d['check'], r['kernels_ms_per_step'])"
done
for m in 1 2; do
  KH_L1R=$m timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py tests/test_gpu_parity.py > "$out/sched_l1r$m.txt" 2>&1 || { echo "tests l1r=$m failed"; tail -20 "$out/sched_l1r$m.txt"; exit 1; }
  tail -1 "$out/sched_l1r$m.txt"
done
