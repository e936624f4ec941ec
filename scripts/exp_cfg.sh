#!/usr/bin/env bash
# A/B of libraries (LIBS) on one config with extra bench args, interleaved, 2 rounds.
# usage: scripts/exp_cfg.sh <config> "<bench args>"
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/cfg
cfg="$1"; args="$2"
for round in 1 2; do
  for lib in $LIBS; do
    tag=$(basename "$lib" .so)
    HRT_LIB="$lib" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --no-golden --steps 2 --warmup 1 $args \
      > "gpurun_out/cfg/${cfg}_$tag.log" 2>&1
    echo "$cfg $tag $(tail -1 gpurun_out/cfg/${cfg}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
