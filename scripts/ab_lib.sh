#!/usr/bin/env bash
# A/B of builds of the library on bench configs, interleaved on one box (2 rounds). LIBS = space-separated
# library paths relative to the package (default "$LIB_A lib/libhrt.so").
# usage: scripts/ab_lib.sh "<bench args>" <config>...
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/ab
args="$1"; shift
libs="${LIBS:-${LIB_A:-} lib/libhrt.so}"
for cfg in "$@"; do
  for round in 1 2; do
    for lib in $libs; do
      tag=$(basename "$lib" .so)
      HRT_LIB="$lib" timeout -k 10 300 python bench.py --config "$cfg" --no-cpu-baseline --no-golden $args \
        > "gpurun_out/ab/${cfg}_$tag.log" 2>&1
      echo "$cfg $tag $(tail -1 gpurun_out/ab/${cfg}_$tag.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], e.get('efficiency', ''), e.get('predicted_ms_per_step', ''))")"
    done
  done
done
