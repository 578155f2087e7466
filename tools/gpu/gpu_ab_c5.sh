#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/c5
for a in "--steps 5 --warmup 2" "--steps 10 --warmup 5" "--steps 5 --warmup 2"; do
  timeout -k 10 300 python -u bench.py $a --no-extras --no-cpu > gpurun_out/c5/run.json 2> gpurun_out/c5/run.err || { tail -20 gpurun_out/c5/run.err; exit 1; }
  python -c "import json;d=json.load(open('gpurun_out/c5/run.json'));print('$a', d['ms_per_step'], d['bbox_extract']['p50_ms'], d['bbox_extract']['p90_ms'])"
done
