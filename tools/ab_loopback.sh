#!/bin/bash
# Same-box A/B of the 8-way loopback per-rank cost: ab/libold.so vs ab/libnew.so, alternated.
set -e
export AMD_SERIALIZE_KERNEL=3
for i in 1 2; do
  for v in old new; do
    KHMER_AMD_LIB=ab/lib$v.so timeout -k 10 200 python3 tools/loopback_bench.py 8 25000000 1 > gpurun_out/abl_${v}_$i.json 2> gpurun_out/abl_${v}_$i.err
  done
done
