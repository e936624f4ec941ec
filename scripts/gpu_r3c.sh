set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3c
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3c/gputest.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config c4 > gpurun_out/r3c/bench_c4.log 2>&1 || exit 1
timeout -k 10 600 python -u bench.py --config c5 --steps 1 --warmup 1 --no-cpu-baseline --no-golden > gpurun_out/r3c/bench_c5.log 2>&1 || exit 1
