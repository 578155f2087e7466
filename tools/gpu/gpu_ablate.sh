#!/bin/bash
# Encode-kernel ablation sweep (FRS_ABLATE bits: 1 fixed slots/no look-back, 2 no CRC, 4 no Rice packing,
# 16 no arena stores); one bench line per setting, no C5 queries, no CPU leg.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/ablate
for a in 0 1 2 4 16 6 23; do
  FRS_ABLATE=$a timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu --queries 0 > gpurun_out/ablate/a$a.log 2>&1 || exit 1
done
echo done
