set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3i
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "tail or stealing or heap or partition" > gpurun_out/r3i/gputest.log 2>&1 || exit 1
for c in c3 c4 c5; do
  for t in 1 0; do
    timeout -k 10 240 python -u bench.py --config $c --steps 3 --warmup 1 --emulate-ranks 0 --tail-split $t --no-cpu-baseline > gpurun_out/r3i/${c}_tail$t.log 2>&1 || exit 1
  done
done
for t in 1 0; do
  timeout -k 10 240 python -u bench.py --config c3 --steps 2 --warmup 1 --emulate-ranks 8 --tail-split $t --no-cpu-baseline > gpurun_out/r3i/c3_split_tail$t.log 2>&1 || exit 1
done
