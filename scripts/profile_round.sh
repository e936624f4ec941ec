#!/usr/bin/env bash
# Round profile of the headline bench (C3): rocprofv3 kernel-trace stats, then the PMC passes (one
# counter group per run, no tracing), summarised for the dominant kernel. Outputs under gpurun_out/<tag>/.
# usage: scripts/profile_round.sh <tag> [bench args...]   (the PMC summary is keyed to the bench line's kernel)
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
tag="$1"; shift
out="gpurun_out/$tag"
mkdir -p "$out"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d "$out/prof" -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --no-golden "$@" > "$out/prof_bench.log" 2>&1
find "$out/prof" -name "*kernel_stats.csv" -exec cp {} "$out/kernel_stats.csv" \;
# (warmup 1: the timed launch deals in the learnt cost order, as the bench's; pmc_summary keeps the timed dispatches)
scripts/pmc.sh "$out/pmc" --no-golden --steps 1 --warmup 1 --emulate-ranks 0 "$@" > "$out/pmc.log" 2>&1
cp "$out/pmc/pmc_summary.json" "$out/pmc_summary.json"
head -4 "$out/kernel_stats.csv"
