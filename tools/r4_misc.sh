#!/bin/bash
# C1's exact command, the genomic nibble fixtures, the tagging end-to-end
# line, then the level-1 A/B and the phase stamps.  Usage: tools/r4_misc.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/r4_$tag
mkdir -p "$out"
true && : \
    ;

timeout -k 10 300 python3 tools/bench_e2e.py --tag --reads 5000000 --cpu-reads 100000 > "$out/e2e_tag.json" 2> "$out/e2e_tag.err" || { tail -5 "$out/e2e_tag.err"; exit 1; }
tail -1 "$out/e2e_tag.json"
bash tools/r4_l1nt.sh "$tag" && bash tools/r4_c4ab.sh "$tag" && bash tools/r4_phases.sh "$tag"
