#!/bin/bash
# serial-frame kernel stats under a list of env settings
set -u
OUT=$1; shift
mkdir -p $OUT; export TMPDIR=/tmp
for s in "$@"; do
  tag=$(echo "$s" | tr ',=/' '___')
  envs=(); [ "$s" != "-" ] && IFS=',' read -ra envs <<< "$s"
  env "${envs[@]}" timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/$tag -o r -- python3 tools/serial_frames.py 20 > $OUT/$tag.log 2>&1 || { tail $OUT/$tag.log; exit 1; }
done
