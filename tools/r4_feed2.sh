#!/bin/bash
# Host feed after the SIMD scan / pack changes: feed and parity tests, then
# end-to-end rates (plain 10M reads; BGZF and gzip 4M reads), packing A/B.
# Usage: tools/r4_feed2.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_feed.py tests/test_gpu_parity.py tests/test_gpu_scripts.py > "$out/tests.txt" 2>&1 || { tail -30 "$out/tests.txt"; exit 1; }
tail -1 "$out/tests.txt"
one() {
  name=$1; shift; envs=$1; shift
  env $envs timeout -k 10 400 python3 tools/bench_e2e.py --cpu-reads 0 --dir /tmp "$@" > "$out/$name.json" 2> "$out/$name.err" || { echo "e2e $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1])
print('$name', '%.3e k-mers/s'%d['value'], '%.2f s'%d['seconds'], 'fastq %.2f GB/s'%d['fastq_GBps'])"
}
one plain10M KH_NONE=0 --reads 10000000 && one plain10M_scalarpack KH_PACK_SCALAR=1 --reads 10000000 &&
one plain10M_b KH_NONE=0 --reads 10000000 && one bgzf4M KH_NONE=0 --reads 4000000 --compress bgzf
