#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Bands (drain fold, four buffers; no auto-steal on covered bands) against the same build without bands
# (lib/libhrt_nob.so, -DHRT_BANDS=0: frame chunks of the whole image) at the same budget; then a kernel-trace
# timeline of C5 at 1024 spp in bands.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
o=gpurun_out/bandab5
mkdir -p $o
run() {  # lib cfg mb tag steps [extra]
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps $5 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
    --no-golden --queue-budget-mb $3 $6 > $o/$2_$3_$4.log 2>&1 || return $?
  echo "$4 $2 $3 $1 $(tail -1 $o/$2_$3_$4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['bands'], d['roofline']['kernel'], d['roofline']['launches_per_step'])")"
}
for round in 1 2; do
  run lib/libhrt.so c3 8192 b$round 3 && run lib/libhrt_nob.so c3 8192 n$round 3 || exit 1
  run lib/libhrt.so c4 8192 b$round 2 && run lib/libhrt_nob.so c4 8192 n$round 2 || exit 1
done
run lib/libhrt.so c5 32768 b1 1 && run lib/libhrt_nob.so c5 32768 n1 1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $o/trace_c5_1024 -o run -- \
  python3 bench.py --config c5 --frames 1024 --steps 1 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
  > $o/trace_c5_1024.log 2>&1 || exit 1
python3 scripts/trace_overlap.py $o/trace_c5_1024 > $o/timeline_c5_1024.txt && tail -3 $o/timeline_c5_1024.txt
