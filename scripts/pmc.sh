#!/usr/bin/env bash
# PMC passes (one counter group per rocprofv3 run, never combined with tracing) over a short bench.
# usage: scripts/pmc.sh <outdir> <bench args...>
set -eu
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
out="$1"; shift
mkdir -p "$out"
i=0
for grp in \
  "SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_INSTS_VALU_FLOPS_FP32 GRBM_GUI_ACTIVE" \
  "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_THREAD_CYCLES_VALU SQ_INSTS_BRANCH SQ_ACTIVE_INST_LDS" \
  "SQ_INSTS_VALU_FMA_F32 SQ_INSTS_VALU_MUL_F32 SQ_INSTS_VALU_ADD_F32 SQ_INSTS_VALU_TRANS_F32 SQ_INST_CYCLES_SMEM SQ_INST_LEVEL_SMEM SQ_LEVEL_WAVES SQ_CYCLES" \
  "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" ; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d "$out" -o "p$i" -- python3 bench.py --no-cpu-baseline "$@" > "$out/p$i.log" 2>&1
done
python3 scripts/pmc_summary.py "$out" ${PMC_KERNEL:-}
