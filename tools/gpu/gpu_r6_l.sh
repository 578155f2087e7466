#!/bin/bash
# round 6 call l: SQ counters and FETCH of the batched decode's kernels (k_sync_count, k_span_crc_lane,
# k_decode_frames_lane) on the C4 arena
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
O=gpurun_out/r6l
mkdir -p $O
D="python3 tools/gpu/dec_bench.py 2 0"
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY --output-format csv -d $O/sqa -o run -- $D > $O/sqa.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_LDS SQ_LDS_IDX_ACTIVE --output-format csv -d $O/sqb -o run -- $D > $O/sqb.log 2>&1 || exit 1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $O/fetch -o run -- $D > $O/fetch.log 2>&1 || exit 1
for k in "k_sync_count<false, true>" k_span_crc_lane k_decode_frames_lane; do echo "## $k"; python3 tools/pmc_by_kernel.py $O/sqa $O/sqb $O/fetch -k $k; done > $O/sq_counters.md 2>&1
cat $O/sq_counters.md
