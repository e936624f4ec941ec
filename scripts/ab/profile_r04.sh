#!/usr/bin/env bash
# Round-4 profiles of C3 / C4 / C5 on the current tree: kernel-trace stats + PMC passes (scripts/profile_round.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
bash scripts/profile_round.sh r04_c3 --config c3 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r04_c4 --config c4 --steps 3 --warmup 1 --emulate-ranks 0 &&
bash scripts/profile_round.sh r04_c5 --config c5 --steps 1 --warmup 1 --emulate-ranks 0
