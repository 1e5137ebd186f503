#!/bin/bash
# Build libmmu_hip.so from git revision $1 into ab/<name>.so (in-tree: it travels to the GPU
# box with gpurun) for same-box A/B timing:  MMU_LIB_PATH=ab/<name>.so python tools/attn_bench.py
set -e
rev=$1; name=${2:-$1}
root=$(git rev-parse --show-toplevel)
tmp=$(mktemp -d)
git -C "$root" archive "$rev" multi-modal-uncertainty_amd/csrc include | tar -x -C "$tmp"
mkdir -p "$root/ab"
make -s -C "$tmp/multi-modal-uncertainty_amd/csrc" -j8 OUT="$root/ab/$name.so" OBJDIR="$tmp/build"
rm -rf "$tmp"
echo "built ab/$name.so from $rev"
