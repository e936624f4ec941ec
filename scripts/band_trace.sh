#!/usr/bin/env bash
# Kernel-trace timestamps of one C4 and one C3 draw in pipelined bands: do consecutive band launches overlap?
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/bandtrace
for cfg in c4 c3; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/bandtrace/$cfg -o run -- \
    python3 bench.py --config $cfg --steps 1 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > gpurun_out/bandtrace/$cfg.log 2>&1 || exit $?
done
