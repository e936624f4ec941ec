#!/usr/bin/env bash
# Round-6 batch L: every job-queue word read before its atomic (HRT_QPEEK=2: lib/libhrt_qpeek2.so, the diagnostic
# lib/libhrt_diag_qpeek2.so) — the C2 tail, then a same-box A/B against the product library on C2 and C3 (8-way emulated
# split on). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06l}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag_qpeek2.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
python3 - "gpurun_out/$tag/wave_tail_c2.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(k, json.dumps({kk: v[kk] for kk in ("trace_ms", "tail_after_first_drain_ms", "end_ms_pcts", "last_job_to_end_ms_pcts")}),
          json.dumps(v["jobs"]["last_5pct_takes"]))
PY
LIBS="lib/libhrt.so lib/libhrt_qpeek2.so" bash scripts/ab_lib.sh "--steps 5" c2 c3 2>&1 | tee "gpurun_out/$tag/ab.txt"
