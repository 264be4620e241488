#!/bin/bash
# A/B of 1024-thread k_scatter_l1f workgroups (KH_L1F_TH) on C2 and C3, with
# the schedule / parity tests under it.  Usage: tools/r4_th.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; cfg=$2; shift 2
  env "$@" timeout -k 10 300 python3 bench.py --config $cfg --steps 3 --cpu-reads 0 --no-unprofiled > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], (d['check'].get('counters_match'), d['check'].get('tables_match')), {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one c2_th512 C2 KH_L1F_TH=512 && one c2_th1024 C2 KH_L1F_TH=1024 &&
one c3_th512 C3 KH_L1F_TH=512 && one c3_th1024 C3 KH_L1F_TH=1024 &&
KH_L1F_TH=1024 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > "$out/sched_th1024.txt" 2>&1 || { tail -20 "$out/sched_th1024.txt"; exit 1; }
tail -1 "$out/sched_th1024.txt"
