#!/bin/bash
# End-of-round check: the whole GPU suite, smoke, the default bench line,
# then every secondary bench line (tools/bench_modes.sh).
# Usage: tools/r4_final2.sh <tag>
set -u
tag=${1:?tag}
cd "$(dirname "$0")/.."
tools/r4_final.sh "$tag" && tools/bench_modes.sh "$tag"
