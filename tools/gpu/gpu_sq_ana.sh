#!/bin/bash
# SQ counters of the C4 step (both kernels; split per kernel by tools/pmc_by_kernel.py) incl. the fp64 issue counts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/sq
mkdir -p $O
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --no-extras --queries 0"
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/a -o run -- $B > $O/a.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $O/b -o run -- $B > $O/b.log 2>&1 || exit 1
for k in k_analyze_v3 k_encode_v3; do echo "== $k"; python3 tools/pmc_by_kernel.py $O/a $O/b -k $k; done
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_FMA_F64 SQ_INSTS_VALU_CVT SQ_INSTS_VALU_INT32 SQ_INSTS_VALU_MUL_F32 --output-format csv -d $O/c -o run -- $B > $O/c.log 2>&1 || { tail -5 $O/c.log; exit 1; }
for k in k_analyze_v3 k_encode_v3; do echo "== $k"; python3 tools/pmc_by_kernel.py $O/c -k $k; done
