#!/bin/bash
# A/B of 2048-record k_scatter_l1f tiles at 4 workgroups per CU (KH_L1F_RPT=4) on C2 and C3, with
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
one c2_rpt8 C2 KH_L1F_RPT=8 && one c2_rpt4 C2 KH_L1F_RPT=4 &&
one c3_rpt8 C3 KH_L1F_RPT=8 && one c3_rpt4 C3 KH_L1F_RPT=4 &&
KH_L1F_RPT=4 timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_schedule.py > "$out/sched_rpt4.txt" 2>&1 || { tail -20 "$out/sched_rpt4.txt"; exit 1; }
tail -1 "$out/sched_rpt4.txt"
