#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ovl
for ab in 0 256 384; do
  FRS_ABLATE=$ab timeout -k 10 300 python bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ovl/ab$ab.log 2>&1 || exit 1
done
echo done
