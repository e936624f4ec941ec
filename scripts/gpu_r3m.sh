set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3m
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3m/$tag.log 2>&1; }
b c4_auto --config c4 --steps 3 || exit 1
b c4_steal --config c4 --steps 3 --steal 2 || exit 1
b c4_steal_jf16 --config c4 --steps 3 --steal 2 --job-frames 16 || exit 1
b c4_steal_jf64 --config c4 --steps 3 --steal 2 --job-frames 64 || exit 1
b c3_steal --config c3 --steps 3 --steal 2 || exit 1
b c5_auto --config c5 --steps 2 || exit 1
b c5_steal --config c5 --steps 2 --steal 2 || exit 1
