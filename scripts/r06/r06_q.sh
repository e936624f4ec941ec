#!/usr/bin/env bash
# (The rt_params.pipeline build it measured was removed after this batch: DESIGN.md §6 Round 6.)
# Round-6 batch Q: kernel timeline of one pipelined C3 step (rocprofv3 kernel trace: start / end of every dispatch).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06q}"
mkdir -p "gpurun_out/$tag"
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for pl in 0 1; do
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "gpurun_out/$tag/p$pl" -o run -- \
    python bench.py --config c3 --no-cpu-baseline --no-golden --steps 2 --warmup 1 --emulate-ranks 0 --pipeline $pl \
    > "gpurun_out/$tag/bench_p$pl.log" 2>&1 || exit 1
done
find "gpurun_out/$tag" -name "*kernel_trace.csv" | sort
