set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3b
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "tris or mixed or mesh or suzanne or fixtures or full_size or sah or heap or partition" > gpurun_out/r3b/gputest.log 2>&1 || exit 1
run() {  # name lib args
  HRT_LIB=$2 timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-golden --emulate-ranks 0 $3 > gpurun_out/r3b/$1.log 2>&1 || return 1
  echo "$1 $(tail -1 gpurun_out/r3b/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'])")"
}
for round in 1 2; do
  run c3_base_$round lib/libhrt.so "--config c3 --steps 3" || exit 1
  run c3_lsph_$round lib/libhrt_l.so "--config c3 --steps 3" || exit 1
  run c4_lds_$round lib/libhrt.so "--config c4 --steps 3" || exit 1
  run c4_off_$round lib/libhrt.so "--config c4 --steps 3 --heap-lds 1" || exit 1
  run c4_uni_$round lib/libhrt_u.so "--config c4 --steps 3" || exit 1
  run c5_lds_$round lib/libhrt.so "--config c5 --frames 256 --steps 2" || exit 1
  run c5_off_$round lib/libhrt.so "--config c5 --frames 256 --steps 2 --heap-lds 1" || exit 1
  run c5_uni_$round lib/libhrt_u.so "--config c5 --frames 256 --steps 2" || exit 1
done
