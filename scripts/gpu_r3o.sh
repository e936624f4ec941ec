set -o pipefail
cd $GRAFT_REPO_ROOT
# phase split of the split kernels (build lib/libhrt_phase.so first: see scripts/phase_split.py)
mkdir -p gpurun_out/r3o
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python -u scripts/phase_split.py --config c3 --frames 1024 --suspend-below 24 > gpurun_out/r3o/c3full.log 2>&1 || exit 1
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python -u scripts/phase_split.py --config c4 --frames 512 > gpurun_out/r3o/c4full.log 2>&1 || exit 1
HRT_LIB=lib/libhrt_phase.so timeout -k 10 300 python -u scripts/phase_split.py --config c5 --frames 16 --suspend-below 32 16 48 > gpurun_out/r3o/c5.log 2>&1 || exit 1
