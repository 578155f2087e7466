#!/bin/bash
# rocprofv3 evidence for the current build: kernel-trace stats, then counter passes (one block per pass)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
B="python3 bench.py --steps 3 --warmup 1 --no-cpu"
timeout -k 10 300 rocprofv3 -L > gpurun_out/prof/counters_list.txt 2>&1 || true
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof/kt -o run -- $B > gpurun_out/prof/kt.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/prof/fetch -o run -- $B > gpurun_out/prof/fetch.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/prof/write -o run -- $B > gpurun_out/prof/write.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/prof/sq1 -o run -- $B > gpurun_out/prof/sq1.log 2>&1 || exit 1
timeout -k 10 400 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS --output-format csv -d gpurun_out/prof/sq2 -o run -- $B > gpurun_out/prof/sq2.log 2>&1 || exit 1
find gpurun_out/prof -name "*.csv" | head -50
echo done
