#!/bin/bash
# Snapshot git revision $1 (package, bench.py, oracle/, tests/, tools/) into ab/<name>/ and
# build its libmmu_hip.so in place: a complete base tree for same-box A/B runs when the
# C-ABI or the Python front-end changed (MMU_LIB_PATH swaps only the library).
set -e
rev=$1; name=${2:-base_tree}
root=$(git rev-parse --show-toplevel)
dst="$root/ab/$name"
rm -rf "$dst"; mkdir -p "$dst"
git -C "$root" archive "$rev" multi-modal-uncertainty_amd include bench.py oracle tests tools pytest.ini | tar -x -C "$dst"
make -s -C "$dst/multi-modal-uncertainty_amd/csrc" -j8 OBJDIR="$dst/build" 2>&1 | grep -v hip-link || true
rm -rf "$dst/build"
echo "tree ab/$name from $rev"
