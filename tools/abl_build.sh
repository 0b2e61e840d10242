#!/bin/bash
# Ablation build of librtx into real-time-ray-tracing_amd/abl_<name>/ (beside lib/, so the data
# path resolves) with extra -D flags; the product build is untouched.
# Usage: tools/abl_build.sh <name> "<-DFLAG ...>"   then RTX_LIB=real-time-ray-tracing_amd/abl_<name>/librtx.so
set -e
D=real-time-ray-tracing_amd/abl_$1
make -s -j8 LIBDIR=$D OBJDIR=$D/obj ABLFLAGS="$2" $D/librtx.so
