#!/bin/bash
# Level-1 path selection: k_scatter_l1f (one launch) against the exact
# two-pass level 1 (KH_L1_EXACT=1) at 358 and 477 buckets (two workgroups
# per CU), C3 under the new default; then the whole GPU suite, smoke and the
# default bench line.  Usage: tools/r4_l1sel.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; shift; envs=$1; shift
  env $envs timeout -k 10 300 python3 bench.py --steps 3 --cpu-reads 0 --no-unprofiled "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], (d['check'].get('counters_match'), d['check'].get('tables_match')), {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one x15_l1f KH_L1_EXACT=0 -x 1.5e9 && one x15_exact KH_L1_EXACT=1 -x 1.5e9 &&
one x20_l1f KH_L1_EXACT=0 -x 2e9 && one x20_exact KH_L1_EXACT=1 -x 2e9 &&
one c3_default KH_L1_EXACT=0 --config C3 || exit 1
timeout -k 10 1500 python3 -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests -m gpu > "$out/gpu_tests.txt" 2>&1 || { grep -E "FAILED|ERROR|Error" "$out/gpu_tests.txt" | head -20; tail -5 "$out/gpu_tests.txt"; exit 1; }
tail -1 "$out/gpu_tests.txt"
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.txt" 2>&1 || { tail -20 "$out/smoke.txt"; exit 1; }
tail -2 "$out/smoke.txt"
timeout -k 10 400 python3 bench.py > "$out/bench.json" 2> "$out/bench.err" || { tail -10 "$out/bench.err"; exit 1; }
tail -1 "$out/bench.json"
