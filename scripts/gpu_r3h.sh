set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3h
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3h/gputest.log 2>&1 || exit 1
bash scripts/profile_round.sh r3h/c3 --emulate-ranks 0 || exit 1
bash scripts/profile_round.sh r3h/c4 --config c4 --emulate-ranks 0 || exit 1
bash scripts/profile_round.sh r3h/c5 --config c5 --emulate-ranks 0 || exit 1
