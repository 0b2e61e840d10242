#!/bin/bash
# Post chain on its own stream (RTX_POST_SPLIT): pipeline / bench-path parity, then bench lines
# with the split off and on.
set -u
O=gpurun_out/r04_split
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread \
    -k "pipeline or bench_path or draw or multirank or denoise" > $O/pytest.log 2>&1 || { tail -30 $O/pytest.log; exit 1; }
tail -1 $O/pytest.log
for r in 1 2; do
  for v in 0 1; do
    RTX_POST_SPLIT=$v timeout -k 10 200 python bench.py --no-cpu-baseline --no-extras --no-self-check > $O/b$v.$r.json 2> $O/b$v.$r.err || { tail -20 $O/b$v.$r.err; exit 1; }
    python -c "import json,sys;d=json.load(open(sys.argv[2]));print('split', sys.argv[1], d['ms_per_step'], d['value'])" $v $O/b$v.$r.json
  done
done
