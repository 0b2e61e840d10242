#!/bin/bash
# Build librtx.so of a committed revision into real-time-ray-tracing_amd/abl_<name>/ (git-ignored,
# beside lib/ so the data path resolves), for same-box A/B runs against the working tree
# (tools/env_ab.sh "RTX_LIB=real-time-ray-tracing_amd/abl_<name>/librtx.so").
# Usage: tools/build_rev.sh <rev> [name]
set -eu
REV=${1:-HEAD}
NAME=${2:-rev}
SRC=/tmp/build_rev_src/$NAME
rm -rf "$SRC" && mkdir -p "$SRC"
git archive "$REV" real-time-ray-tracing_amd/csrc include | tar -x -C "$SRC"
OUT=real-time-ray-tracing_amd/abl_$NAME
mkdir -p "$OUT"
make -s -j8 CSRC="$SRC/real-time-ray-tracing_amd/csrc" LIBDIR="$OUT" OBJDIR="/tmp/build_rev_obj/$NAME" "$OUT/librtx.so"
echo "built $OUT/librtx.so from $(git rev-parse --short "$REV")"
