#!/bin/bash
# round 6 call r: analysis / encode kernel time against the tile count (C4 width, 26 / 52 / 79 tile rows): is there
# a partial last round of waves?
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6r
mkdir -p $O
for h in 13312 26624 40000 19968 33280; do
  timeout -k 10 200 python -u bench.py --height $h --no-extras --no-cpu --queries 0 --steps 10 > $O/h$h.json 2> $O/h$h.err || { tail -20 $O/h$h.err; exit 1; }
  python -c "
import json;d=json.loads(open('$O/h$h.json').read().strip().splitlines()[-1])
print($h, d['config']['tiles'], d['ms_per_step'], d['kernels_ms'])"
done
