#!/usr/bin/env bash
# Round-6 closing profiles of the final tree: rocprofv3 kernel-trace stats and the PMC passes (timed dispatches only,
# scripts/pmc_summary.py) for C3 / C4 / C5, the compiler resource usage, then the GPU suite and the default bench line.
# Logs: gpurun_out/r06_*.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
bash scripts/profile_round.sh r06_c3 --config c3 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r06_c4 --config c4 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r06_c5 --config c5 --steps 1 --warmup 1 --emulate-ranks 0 &&
for c in c3 c4 c5; do python3 -c "
import json; s=json.load(open('gpurun_out/r06_$c/pmc_summary.json'))
print('$c', s['_kernels'], s['_dispatches_per_pass'].get('FETCH_SIZE'), round(s['hbm_bytes_per_launch']/1e9,3), 'GB/launch',
      round(s['SQ_THREAD_CYCLES_VALU']/s['SQ_ACTIVE_INST_VALU'],2), 'lanes')"; done
