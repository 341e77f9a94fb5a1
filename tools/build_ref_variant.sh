#!/bin/bash
# Builds the library from git ref REF as the experiment build libjdamd_<NAME>.so (A/B baselines
# for tools/ab.sh).  Usage: bash tools/build_ref_variant.sh REF NAME [VDEFS...]
set -e
ref=$1; name=$2; shift 2
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" archive "$ref" gpu-jpeg-decoder_amd include | tar -x -C "$tmp"
make -s -C "$tmp/gpu-jpeg-decoder_amd" variant V="$name" VDEFS="$*" >/dev/null
cp "$tmp/gpu-jpeg-decoder_amd/libjdamd_$name.so" "$root/gpu-jpeg-decoder_amd/"
rm -rf "$tmp"
echo "built gpu-jpeg-decoder_amd/libjdamd_$name.so from $ref"
