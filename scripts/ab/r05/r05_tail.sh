#!/usr/bin/env bash
# Round-5 diagnosis of short launches and of C3's walk lanes (diagnostic build lib/libhrt_diag.so): per-wave records of a
# 1/8 C4 share and the full image (scripts/wave_tail.py), the walk's lane counters on C3 (scripts/diag_split.py), and the
# C2 8-way emulated split by job size. Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../../..}"
tag="${1:-r05b}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so bash scripts/gpu_step.sh "$tag/wave_tail_c4" 300 python scripts/wave_tail.py --config c4 --ranks 8 --rank 4 0 7 --full \
  --- "$tag/wave_tail_c3" 300 python scripts/wave_tail.py --config c3 --ranks 8 --rank 4 --full \
  --- "$tag/diag_split_c3" 300 python scripts/diag_split.py --suspend 16 24 32 48 --frames 64
for jf in 4 8 16; do
  bash scripts/gpu_step.sh "$tag/c2_jf$jf" 300 python bench.py --config c2 --no-cpu-baseline --no-golden --steps 5 --job-frames $jf || exit 1
  tail -1 "gpurun_out/$tag/c2_jf$jf.log" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); e=d['emulated_split']; print('c2 jf $jf', d['value'], d['ms_per_step'], e['efficiency'], e['predicted_ms_per_step'])"
done
