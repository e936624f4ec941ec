set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3a
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3a/gputest.log 2>&1 &&
timeout -k 10 300 python -u bench.py > gpurun_out/r3a/bench_c3.log 2>&1 &&
timeout -k 10 200 python -u bench.py --emulate-ranks 8 --row-block 1 --no-cpu-baseline --no-golden --steps 2 > gpurun_out/r3a/bench_c3_rb1.log 2>&1 &&
timeout -k 10 200 python -u bench.py --emulate-ranks 4 --no-cpu-baseline --no-golden --steps 2 > gpurun_out/r3a/bench_c3_e4.log 2>&1 &&
timeout -k 10 200 python -u bench.py --emulate-ranks 2 --no-cpu-baseline --no-golden --steps 2 > gpurun_out/r3a/bench_c3_e2.log 2>&1 &&
timeout -k 10 400 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-golden > gpurun_out/r3a/bench_c5.log 2>&1
