set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3u
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "mixed or heap or fixtures or stealing or full_size or bvh" > gpurun_out/r3u/gputest.log 2>&1 || exit 1
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3u/$tag.log 2>&1; }
for k in 1 2; do
b c5_sel1_$k --config c5 --steps 1 --frames 1024 || exit 1
HRT_LIB=lib/libhrt_sel0.so b c5_sel0_$k --config c5 --steps 1 --frames 1024 || exit 1
done
