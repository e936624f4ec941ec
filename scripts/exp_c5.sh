#!/usr/bin/env bash
# C5 at 256 spp for A/B of libraries and suspend thresholds: LIBS x thresholds.
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/c5
for lib in $LIBS; do
  for sb in "$@"; do
    tag=$(basename "$lib" .so)_$sb
    HRT_LIB="$lib" timeout -k 10 200 python bench.py --config c5 --frames 256 --no-cpu-baseline --no-golden --steps 2 --warmup 1 \
      --suspend-below "$sb" > "gpurun_out/c5/$tag.log" 2>&1
    echo "c5 $tag $(tail -1 gpurun_out/c5/$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
