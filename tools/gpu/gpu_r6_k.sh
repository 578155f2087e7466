#!/bin/bash
# round 6 call k: the default bench line's counter fields with the committed summary of this build
set -o pipefail
mkdir -p gpurun_out/r6k
timeout -k 10 300 python bench.py --no-extras --no-cpu > gpurun_out/r6k/bench.json 2> gpurun_out/r6k/bench.err
rc=$?
tail -3 gpurun_out/r6k/bench.err
python -c "
import json; d=json.loads(open('gpurun_out/r6k/bench.json').read().strip().splitlines()[-1])
print(d['ms_per_step'], json.dumps(d['roofline']))"
exit $rc
