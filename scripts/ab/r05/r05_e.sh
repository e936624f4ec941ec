#!/usr/bin/env bash
# Round-5 batch E: C4's 8-way emulated split under the short-launch options (bench.py knobs apply to the full image and
# to every share): stealing auto (default), stealing off (the tail split then applies), off + eighths, 16-frame jobs.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05e}"
mkdir -p "gpurun_out/$tag"
for v in "auto:" "nosteal:--steal 1" "nosteal8:--steal 1 --tail-split 3" "jf16:--job-frames 16" "jf16nosteal:--job-frames 16 --steal 1"; do
  name="${v%%:*}"; args="${v#*:}"
  bash scripts/gpu_step.sh "$tag/c4_$name" 300 python bench.py --config c4 --no-cpu-baseline --no-golden --steps 3 $args || exit 1
  tail -1 "gpurun_out/$tag/c4_$name.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['emulated_split']; print('c4 $name', d['value'], d['ms_per_step'], e['efficiency'], e['predicted_ms_per_step'], [r['ms_per_step'] for r in e['per_rank']])"
done
# the wave records of the default (stealing) and the tail-split configurations of a 1/8 C4 share
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --full \
  --- "$tag/wave_tail_c4_nosteal" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 --steal 1
