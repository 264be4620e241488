#!/bin/bash
# A/B of level-1 tables per launch (KH_L1_NT: with launch windows each launch
# holds only its tables' buckets) and 4 workgroups per CU (abx/libwpe8.so,
# <= 64 VGPRs) on the C2 bench.  Usage: tools/r4_l1nt.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
one() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 3 --cpu-reads 0 --no-unprofiled > "$out/$name.json" 2> "$out/$name.err" || { echo "bench $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1]); r=d['roofline']
print('$name', round(d['ms_per_step'],1), 'ms/step', '%.3e'%d['value'], d['check'].get('counters_match'), d['check'].get('tables_match'), {k:v for k,v in r['kernels_ms_per_step'].items() if v>1})"
}
one base KH_L1_NT=8 &&
one nt2 KH_L1_NT=2 &&
one nt1 KH_L1_NT=1 &&
one wpe8_nt2_w4 KHMER_AMD_LIB=abx/libwpe8.so KH_L1_NT=2 KH_L1F_WPC=4 &&
one wpe8_nt8_w3 KHMER_AMD_LIB=abx/libwpe8.so KH_L1_NT=8 &&
one base2 KH_L1_NT=8
