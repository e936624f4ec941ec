set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3t
b() { tag=$1; shift; timeout -k 10 240 python -u bench.py --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden "$@" > gpurun_out/r3t/$tag.log 2>&1; }
for sb in 24 32 40 48; do b c4_sb$sb --config c4 --steps 3 --suspend-below $sb || exit 1; done
for sb in 32 40 48 56; do b c5_sb$sb --config c5 --steps 1 --frames 1024 --suspend-below $sb || exit 1; done
