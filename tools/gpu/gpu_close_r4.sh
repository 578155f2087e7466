#!/bin/bash
# Round-4 closing call: GPU suite + smoke + default bench line, then the rocprofv3 profile of the same library
# (kernel stats, FETCH/WRITE/VALU passes stamped with the library hash, SQ counters).
set -o pipefail
cd "$GRAFT_REPO_ROOT"
./tools/gpu/gpu_final_r4.sh && ./tools/gpu/gpu_prof_r4.sh
