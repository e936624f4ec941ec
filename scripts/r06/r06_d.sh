#!/usr/bin/env bash
# Round-6 batch D: the round-6 tree (packet off by default; k_trace_split's rank by mbcnt and its query count per wave)
# against the round-5 library (lib/libhrt_r05.so, built from HEAD~ sources) on C3 / C4, same box, interleaved; then the
# GPU suite. Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06d}"
mkdir -p "gpurun_out/$tag"
for cfg in c3 c4; do
  for round in 1 2; do
    for lib in lib/libhrt_r05.so lib/libhrt.so; do
      log="gpurun_out/$tag/${cfg}_$(basename $lib .so)_$round.log"
      HRT_LIB="$lib" timeout -k 10 300 python bench.py --config $cfg --steps 5 --no-cpu-baseline --no-golden > "$log" 2>&1 || exit 1
      echo "$cfg $lib round $round: $(tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "gpurun_out/$tag/ab.txt"
    done
  done
done
bash scripts/gpu_step.sh "$tag/gputest" 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread
