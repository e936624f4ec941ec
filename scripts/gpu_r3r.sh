set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3r
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed or heap or large_mesh or fixtures or stealing or tail or full_size" > gpurun_out/r3r/gputest.log 2>&1 || exit 1
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3r/$tag.log 2>&1; }
b c5_split --config c5 --steps 2 || exit 1
HRT_LIB=lib/libhrt_ms0.so b c5_base --config c5 --steps 2 || exit 1
