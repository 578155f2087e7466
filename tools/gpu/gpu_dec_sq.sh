#!/bin/bash
# SQ counters of the decode kernels per variant library (variants/lib<name>.so): one --pmc pass each
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/decsq
cd /tmp
for v in ${VARIANTS:-dec_b8}; do
  FRS_LIB_PATH=$GRAFT_REPO_ROOT/variants/lib$v.so timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR -d $GRAFT_REPO_ROOT/gpurun_out/decsq/$v -o pmc -- python3 $GRAFT_REPO_ROOT/tools/gpu/dec_bench.py 1 0 > /dev/null 2> $GRAFT_REPO_ROOT/gpurun_out/decsq/$v.err || { tail -5 $GRAFT_REPO_ROOT/gpurun_out/decsq/$v.err; exit 1; }
done
echo sq done
