#!/bin/bash
# Build an ablation variant of librtx.so: copy the sources to /tmp, apply the sed expressions to
# the named csrc files, build into real-time-ray-tracing_amd/abl_<name>/librtx.so (in-tree so the
# data directory resolves and it travels to the GPU box; git-ignored).
# Usage: tools/ablate.sh <name> "<file>:<sed expr>" ...
set -eu
NAME=$1; shift
SRC=/tmp/ablate_src/$NAME
rm -rf "$SRC"; mkdir -p "$SRC/real-time-ray-tracing_amd"
cp -r real-time-ray-tracing_amd/csrc "$SRC/real-time-ray-tracing_amd/"
cp -r include "$SRC/"
for spec in "$@"; do
  f=${spec%%:*}; e=${spec#*:}
  sed -i "$e" "$SRC/real-time-ray-tracing_amd/csrc/$f"
done
OUT=real-time-ray-tracing_amd/abl_$NAME
mkdir -p "$OUT"
make -s -j8 CSRC="$SRC/real-time-ray-tracing_amd/csrc" LIBDIR="$OUT" OBJDIR="/tmp/ablate_obj/$NAME" "$OUT/librtx.so"
echo "built $OUT/librtx.so"
