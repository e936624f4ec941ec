set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3g
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread -k "heap or stealing or mixed or suzanne or mesh" > gpurun_out/r3g/gputest.log 2>&1 || exit 1
run() {  # name args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-golden --emulate-ranks 0 $2 > gpurun_out/r3g/$1.log 2>&1 || return 1
  echo "$1 $(tail -1 gpurun_out/r3g/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['kernel'])")"
}
for round in 1 2; do
  for h in 2 3 4; do
    run c4_h${h}_$round "--config c4 --steps 3 --heap-lds $h" || exit 1
    run c5_h${h}_$round "--config c5 --frames 256 --steps 2 --heap-lds $h" || exit 1
  done
done
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python -u scripts/diag_split.py --suspend 24 --frames 64 > gpurun_out/r3g/diag_c3.log 2>&1 || exit 1
