#!/usr/bin/env bash
# Round-6 batch B: the packet walk (all lanes in the walk, large list after it, 7 waves) — GPU suite, then a same-box
# A/B on C3: packet off / on (product library) and on at 6 waves (lib/libhrt_p6.so). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06b}"
mkdir -p "gpurun_out/$tag"
bash scripts/gpu_step.sh "$tag/gputest" 1000 python -u -m pytest tests -m gpu -x -v --timeout 240 --timeout-method thread || exit 1
grep -q " passed" "gpurun_out/$tag/gputest.log" && ! grep -q "FAILED\|ERROR" "gpurun_out/$tag/gputest.log" || exit 1
for round in 1 2; do
  for v in "lib/libhrt.so 1" "lib/libhrt.so 2" "lib/libhrt_p6.so 2"; do
    set -- $v
    log="gpurun_out/$tag/c3_$(basename $1 .so)_p$2_$round.log"
    HRT_LIB="$1" timeout -k 10 300 python bench.py --config c3 --steps 5 --no-cpu-baseline --no-golden --packet "$2" > "$log" 2>&1 || exit 1
    echo "c3 $1 packet $2 round $round: $(tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "gpurun_out/$tag/ab.txt"
  done
done
