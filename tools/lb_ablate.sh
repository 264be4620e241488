#!/bin/bash
# Per-rank cost of the 8-way sharded level 1 (loopback) under timing
# ablations of k_own_l1f (KH_ABLATE 64: no bucket placement, 128: no
# ownership test), with and without table_mod's f64 quotient (KH_FASTMOD),
# and one SQ counter pass over k_own_l1f.
set -e
export AMD_SERIALIZE_KERNEL=3
for fm in 1 0; do
  for ab in 0 64 128; do
    KH_FASTMOD=$fm KH_ABLATE=$ab timeout -k 10 200 python3 tools/loopback_bench.py 8 25000000 1 > gpurun_out/lb_fm${fm}_ab$ab.json 2> gpurun_out/lb_fm${fm}_ab$ab.err
  done
done
export TMPDIR=/tmp
timeout -s KILL 150 rocprofv3 --kernel-include-regex own_l1f --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU -d gpurun_out/lb_pmc -o run --output-format csv -- python3 tools/loopback_bench.py 8 10000000 1 > gpurun_out/lb_pmc.json 2> gpurun_out/lb_pmc.err
