set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3v
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "golden or bvh or split or tail or partition or full_size" > gpurun_out/r3v/gputest.log 2>&1 || exit 1
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3v/$tag.log 2>&1; }
for k in 1 2 3; do
b c3_ka_$k --config c3 --steps 3 || exit 1
HRT_LIB=lib/libhrt_base.so b c3_base_$k --config c3 --steps 3 || exit 1
done
