#!/bin/bash
# Round-6 per-rank model lines (tools/rank_model.py) on the final kernels:
# C2 / C4 weak scaling in delta mode (sparse deltas probed), C4 strong
# scaling (6.25M reads a rank) in both modes.  Usage: tools/r6_models.sh <tag>
set -o pipefail
tag=${1:?tag}
cd "$(dirname "$0")/.."
out=gpurun_out/$tag; mkdir -p $out
run() {
    name=$1; shift
    timeout -k 10 500 python3 -u tools/rank_model.py "$@" > $out/$name.json 2> $out/$name.err || { echo "FAIL $name"; tail -5 $out/$name.err; return 1; }
    python3 -c "import json,sys; d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1]); print(sys.argv[2], d['compute_ms_per_rank_step'], d['wire_ms_at_assumed_rate'], d['rank_step_ms_unoverlapped'], d.get('delta_sparse_ratio'), d.get('rank_step_ms_sparse_unoverlapped'))" $out/$name.json $name
}
run c2_delta --mode delta --world 8 --config C2 &&
run c4_delta --mode delta --world 8 --config C4 --batch-kmers 2400000000 &&
run c4s_delta --mode delta --world 8 --config C4 --reads 6250000 &&
run c4s_exchange --mode exchange --world 8 --config C4 --reads 6250000
