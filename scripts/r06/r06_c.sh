#!/usr/bin/env bash
# Round-6 batch C: why the C3 packet walk is slower — phase split of k_trace_split with packet off / on (diagnostic phase
# build), and a same-box A/B of packet off / on against the packet kernel without its walk (lib/libhrt_pdry.so: the
# PACKET instantiation's register allocation alone). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06c}"
mkdir -p "gpurun_out/$tag"
for p in 1 2; do
  HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python scripts/phase_split.py --config c3 --frames 16 --packet $p \
    >> "gpurun_out/$tag/phase_c3.log" 2>&1 || exit 1
done
cat "gpurun_out/$tag/phase_c3.log"
for round in 1 2; do
  for v in "lib/libhrt.so 1" "lib/libhrt.so 2" "lib/libhrt_pdry.so 2"; do
    set -- $v
    log="gpurun_out/$tag/c3_$(basename $1 .so)_p$2_$round.log"
    HRT_LIB="$1" timeout -k 10 300 python bench.py --config c3 --steps 5 --no-cpu-baseline --no-golden --packet "$2" > "$log" 2>&1 || exit 1
    echo "c3 $1 packet $2 round $round: $(tail -1 "$log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")" | tee -a "gpurun_out/$tag/ab.txt"
  done
done
