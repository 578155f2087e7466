#!/bin/bash
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/fused
FRS_FUSED=1 FRS_ANA_DBG=1 timeout -k 10 60 python -u tools/gpu/dbg_fused.py > gpurun_out/fused/dbg.log 2>&1; rc=$?
cat gpurun_out/fused/dbg.log
exit $rc
