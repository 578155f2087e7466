#!/bin/bash
# One SQ counter pass (LDS conflicts, instruction mix) per library variant: variants/libhead.so, variants/libnew.so.
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
rm -rf gpurun_out/sq3; mkdir -p gpurun_out/sq3
B="python3 bench.py --steps 2 --warmup 1 --no-cpu --queries 0"
for n in head new; do
  FRS_LIB_PATH=$PWD/variants/lib$n.so timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU --output-format csv -d gpurun_out/sq3/$n -o run -- $B > gpurun_out/sq3/$n.log 2>&1 || exit 1
  python3 tools/pmc_summary.py gpurun_out/sq3/$n > gpurun_out/sq3/sum_$n.md || exit 1
done
echo done
