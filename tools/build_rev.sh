#!/bin/bash
# Build libsurfhip.so of a git revision into cuda-surf_amd/diag/<name>/ (for
# tools/ab.sh A/B against the working tree):  bash tools/build_rev.sh <rev> <name>
set -eu
REV=$1; NAME=$2
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
T=$(mktemp -d)
git -C "$ROOT" archive "$REV" cuda-surf_amd/csrc include cuda-surf_amd/Makefile | tar -x -C "$T"
make -s -C "$T/cuda-surf_amd" libsurfhip.so
mkdir -p "$ROOT/cuda-surf_amd/diag/$NAME"
cp "$T/cuda-surf_amd/libsurfhip.so" "$ROOT/cuda-surf_amd/diag/$NAME/"
rm -rf "$T"
echo "built $REV -> cuda-surf_amd/diag/$NAME"
