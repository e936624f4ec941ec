set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3n
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3n/gputest.log 2>&1 || exit 1
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3n/$tag.log 2>&1; }
b c3 --config c3 --steps 3 --emulate-ranks 8 || exit 1
b c4 --config c4 --steps 3 --emulate-ranks 8 || exit 1
b c2 --config c2 --steps 3 --emulate-ranks 0 || exit 1
