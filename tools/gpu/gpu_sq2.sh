#!/bin/bash
# SQ counter passes on the encode path for the full kernel and the FRS_ABLATE=23 core (no look-back, CRC,
# packing, stores): instruction mix, busy/wait cycles, LDS bank conflicts.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/sq2
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --queries 0"
for a in 0 23; do
  FRS_ABLATE=$a timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d gpurun_out/sq2/a$a -o run -- $B > gpurun_out/sq2/a$a.log 2>&1 || exit 1
  FRS_ABLATE=$a timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA --output-format csv -d gpurun_out/sq2/b$a -o run -- $B > gpurun_out/sq2/b$a.log 2>&1 || exit 1
done
python3 tools/pmc_summary.py gpurun_out/sq2/a0 gpurun_out/sq2/b0 > gpurun_out/sq2/sum0.md
python3 tools/pmc_summary.py gpurun_out/sq2/a23 gpurun_out/sq2/b23 > gpurun_out/sq2/sum23.md
echo done
