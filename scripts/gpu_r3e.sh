set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3e
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "stealing or partition or heap or fixtures" > gpurun_out/r3e/gputest.log 2>&1 || exit 1
run() {  # name lib args
  HRT_LIB=$2 timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-golden $3 > gpurun_out/r3e/$1.log 2>&1 || return 1
  echo "$1 $(tail -1 gpurun_out/r3e/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], d['roofline']['kernel'], e.get('efficiency'), e.get('predicted_ms_per_step'))")"
}
for round in 1 2; do
  run c3_ref_$round lib/libhrt_ref.so "--config c3 --steps 3 --emulate-ranks 8" || exit 1
  run c3_steal_$round lib/libhrt.so "--config c3 --steps 3 --emulate-ranks 8" || exit 1
  run c3_nosteal_$round lib/libhrt.so "--config c3 --steps 3 --emulate-ranks 8 --steal 1" || exit 1
  run c4_ref_$round lib/libhrt_ref.so "--config c4 --steps 3 --emulate-ranks 8" || exit 1
  run c4_steal_$round lib/libhrt.so "--config c4 --steps 3 --emulate-ranks 8" || exit 1
  run c5_ref_$round lib/libhrt_ref.so "--config c5 --frames 256 --steps 2 --emulate-ranks 0" || exit 1
  run c5_steal_$round lib/libhrt.so "--config c5 --frames 256 --steps 2 --emulate-ranks 0" || exit 1
done
