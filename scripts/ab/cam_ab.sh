#!/usr/bin/env bash
# (The scalar row quotient, global_row8, measured no gain and was removed; profiles/r04/so/cam_ab.txt.)
# Primary-ray generation: the fast exact px / wm1, py / hm1 and v / |v| of the sphere program (lib/libhrt_cam.so, kept), and
# with them the tile's global rows from a scalar quotient (global_row8; lib/libhrt.so), against commit 606b7ce
# (lib/libhrt_base.so): the GPU suite, then interleaved C3, C2 and C4 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/cam_ab
mkdir -p $o
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib cfg tag
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config $2 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > $o/$2_$3.log 2>&1 || return $?
  echo "$3 $2 $(tail -1 $o/$2_$3.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
}
for round in 1 2 3; do
  run lib/libhrt_base.so c3 base$round && run lib/libhrt_cam.so c3 cam$round && run lib/libhrt.so c3 row$round || exit 1
done
for round in 1 2; do
  run lib/libhrt_base.so c2 base$round && run lib/libhrt_cam.so c2 cam$round && run lib/libhrt.so c2 row$round || exit 1
done
for round in 1 2; do
  run lib/libhrt_cam.so c4 cam$round && run lib/libhrt.so c4 row$round || exit 1
done
