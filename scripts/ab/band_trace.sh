#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Kernel-trace timestamps of one C4 and one C3 draw (sample buffer): with a budget below the draw's colours the
# draw runs as pipelined bands — do consecutive band launches overlap, and how long are their drains?
# usage: scripts/band_trace.sh [budget MiB] [tag]
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
budget="${1:-8192}"; tag="${2:-b$budget}"
mkdir -p gpurun_out/bandtrace
for cfg in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bandtrace/${tag}_$cfg -o run -- \
    python3 bench.py --config $cfg --steps 1 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    --queue-budget-mb "$budget" > gpurun_out/bandtrace/${tag}_$cfg.log 2>&1 || exit $?
done
