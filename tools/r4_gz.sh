#!/bin/bash
# Compressed-input feed: the parity tests, then end-to-end consume_seqfile
# rates (C2-shaped Countgraph, tools/bench_e2e.py) for plain, gzip and BGZF
# input, serial inflate (KH_ASYNC_INFLATE=0) against the threaded one, and
# BGZF streamed through one parser (KH_BGZF_CHUNKED=0) or chunk-parallel.
# Usage: tools/r4_gz.sh <tag> [reads]
set -u
tag=${1:?tag}; reads=${2:-2000000}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
d=$(mktemp -d /tmp/khgz.XXXX)
trap 'rm -rf "$d"' EXIT
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_feed.py > "$out/feed_tests.txt" 2>&1 || { tail -30 "$out/feed_tests.txt"; exit 1; }
tail -1 "$out/feed_tests.txt"
for c in none gzip bgzf; do
  timeout -k 10 300 python3 tools/bench_e2e.py --reads $reads --make $d/$c.fq --compress $c > "$out/make_$c.json" || exit 1
  cat "$out/make_$c.json"
done
run() {
  name=$1; async=$2; f=$3; chunked=${4:-1}
  KH_BGZF_CHUNKED=$chunked KH_ASYNC_INFLATE=$async timeout -k 10 400 python3 tools/bench_e2e.py --reads $reads --cpu-reads 0 --input $f > "$out/$name.json" 2> "$out/$name.err" || { echo "e2e $name failed"; tail -5 "$out/$name.err"; return 1; }
  python3 -c "
import json; d=json.loads(open('$out/$name.json').read().strip().splitlines()[-1])
print('$name', '%.3e k-mers/s'%d['value'], '%.2f s'%d['seconds'], 'fastq %.2f GB/s'%d['fastq_GBps'], 'file %.3f GB/s'%d['file_GBps'])"
}
run plain 1 $d/none.fq &&
run gzip_serial 0 $d/gzip.fq.gz && run gzip_async 1 $d/gzip.fq.gz &&
run bgzf_serial 0 $d/bgzf.fq.bgz && run bgzf_stream 1 $d/bgzf.fq.bgz 0 && run bgzf_chunked 1 $d/bgzf.fq.bgz 1
