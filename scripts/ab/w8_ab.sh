#!/usr/bin/env bash
# C3 at 8 waves per SIMD (lib/libhrt_w8.so: 64 VGPRs, 6-float frame-block entries with the RNG state recomputed,
# 160-node LDS cap) against 7 waves (lib/libhrt.so): sphere parity tests on the 8-wave build, then C3 lines.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
o=gpurun_out/w8_ab
mkdir -p $o
HRT_LIB=lib/libhrt_w8.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread \
  -k "c3 or sphere or golden or schedule or tail or count or steal or suspend" > $o/gputest.log 2>&1 || { tail -30 $o/gputest.log; exit 1; }
tail -1 $o/gputest.log
run() {  # lib tag
  HRT_LIB=$1 timeout -k 10 300 python bench.py --config c3 --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    > $o/c3_$2.log 2>&1 || return $?
  echo "$2 $(tail -1 $o/c3_$2.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'])")"
}
for round in 1 2 3; do
  run lib/libhrt.so w7_$round && run lib/libhrt_w8.so w8_$round || exit 1
done
