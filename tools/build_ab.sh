#!/bin/bash
# Build the batch library of another git revision into k2hash_amd/lib/ab/<name>/ so that
# tools/ab_libs.py can time it against the working tree in ONE process (interleaved).
#   bash tools/build_ab.sh <git-rev> [name]
set -eo pipefail
REV=${1:?git rev}; NAME=${2:-$REV}
ROOT=$(cd "$(dirname "$0")/.." && pwd)
WT=$(mktemp -d /tmp/k2h_ab.XXXXXX)
git -C "$ROOT" archive "$REV" k2hash_amd/csrc include | tar -x -C "$WT"
make -C "$WT/k2hash_amd/csrc" -j8 >/dev/null
mkdir -p "$ROOT/k2hash_amd/lib/ab/$NAME"
cp "$WT/k2hash_amd/lib/libk2hash_amd.so" "$ROOT/k2hash_amd/lib/ab/$NAME/"
rm -rf "$WT"
echo "$ROOT/k2hash_amd/lib/ab/$NAME/libk2hash_amd.so"
