set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3x
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3x/gputest.log 2>&1 || exit 1
bash scripts/profile_round.sh r3x/c3 --emulate-ranks 0 || exit 1
bash scripts/profile_round.sh r3x/c4 --config c4 --emulate-ranks 0 || exit 1
bash scripts/profile_round.sh r3x/c5 --config c5 --emulate-ranks 0 --steps 1 --warmup 0 || exit 1
