#!/usr/bin/env bash
# Round-5 closing profiles: rocprofv3 kernel-trace stats + the PMC passes (scripts/profile_round.sh) of C3 / C4 / C5 on
# the final tree.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile_round.sh r05p_c3 --config c3 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r05p_c4 --config c4 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r05p_c5 --config c5 --steps 1 --warmup 1 --emulate-ranks 0
