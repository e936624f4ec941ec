#!/usr/bin/env bash
# Round-6 batch H: the job queue read before a foreign XCD queue's atomic (HRT_QPEEK) — the C2 tail in the diagnostic
# build, then a same-box A/B against the library without it (lib/libhrt_qpeek0.so) on C2 / C3 / C4 with the bench's
# 8-way emulated split. Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06h}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
python3 - "gpurun_out/$tag/wave_tail_c2.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(k, json.dumps({kk: v[kk] for kk in ("trace_ms", "tail_after_first_drain_ms", "last_job_to_end_ms_pcts", "clk_per_round_last_job_pcts")}),
          json.dumps(v["jobs"]["last_5pct_takes"]))
PY
LIBS="lib/libhrt_qpeek0.so lib/libhrt.so" bash scripts/ab_lib.sh "--steps 5" c2 c3 c4 2>&1 | tee "gpurun_out/$tag/ab.txt"
