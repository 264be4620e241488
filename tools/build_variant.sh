#!/bin/bash
# Development: build libkhmer_hip.so from the current sources with extra
# compiler flags into ab/lib<name>.so (select it on the GPU box with
# KHMER_AMD_LIB=ab/lib<name>.so, e.g. through tools/ab_multi.sh).
# Usage: tools/build_variant.sh <name> "<extra hipcc flags>"
set -euo pipefail
name=${1:?name}; flags=${2:-}
root="$(cd "$(dirname "$0")/.." && pwd)"
tmp=/tmp/kh_variant_$name
rm -rf "$tmp"; mkdir -p "$tmp/khmer_amd" "$root/${KH_VARIANT_DIR:-ab}"
cp -r "$root/include" "$tmp/include"
cp -r "$root/khmer_amd/csrc" "$tmp/khmer_amd/csrc"
rm -rf "$tmp/khmer_amd/csrc/build"
make -s -C "$tmp/khmer_amd/csrc" -j4 OUT="$root/${KH_VARIANT_DIR:-ab}/lib$name.so" EXTRA_HIPFLAGS="$flags"
echo "built ${KH_VARIANT_DIR:-ab}/lib$name.so"
