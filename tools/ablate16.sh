#!/bin/bash
# The --ablate 16 run (level-1 record writes skipped: timing only, results
# wrong by design) on a -DKH_ABLATE development build (tools/build_variant.sh
# ablate -DKH_ABLATE, KH_VARIANT_DIR=var), C2 and C4 (near-prime level 1) and C2 with the per-table level 1
# (KH_NEAR_PRIME=0, k_scatter_l1p).  Usage: tools/ablate16.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
mkdir -p gpurun_out/$tag
for cfg in C2 C4 C2-l1p; do
    np=1; [ $cfg = C2-l1p ] && np=0
    KH_NEAR_PRIME=$np KHMER_AMD_LIB=var/libablate.so timeout -k 10 300 python -u bench.py --config ${cfg%-l1p} --ablate 16 --steps 2 --warmup 1 \
        --cpu-reads 0 --no-unprofiled > gpurun_out/$tag/ab16_$cfg.json 2> gpurun_out/$tag/ab16_$cfg.err
    rc=$?
    echo "ablate16 $cfg rc=$rc"; tail -2 gpurun_out/$tag/ab16_$cfg.err
    [ $rc -eq 0 ] || exit 1
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(round(d['ms_per_step'],1), d['roofline']['kernels_ms_per_step'])" gpurun_out/$tag/ab16_$cfg.json
done
