#!/usr/bin/env bash
# Round-6 batch K: slow waves retire near the launch's end (HRT_RETIRE, k_trace) — the C2 tail in the diagnostic build,
# C2 parity tests on the product build, then a same-box A/B against lib/libhrt_retire0.so (C2 full image with the bench's
# 8-way emulated split). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06k}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
python3 - "gpurun_out/$tag/wave_tail_c2.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(k, json.dumps({kk: v[kk] for kk in ("trace_ms", "tail_after_first_drain_ms", "end_ms_pcts", "last_job_to_end_ms_pcts", "jobs_per_wave_pcts")}))
PY
timeout -k 10 400 python -u -m pytest tests/test_gpu_timed.py::test_c2_as_timed tests/test_gpu_parity.py -x -q --timeout 300 \
  --timeout-method thread -k "c2 or C2 or sample_queue or golden or draw_frames" > "gpurun_out/$tag/tests.log" 2>&1 || { tail -30 "gpurun_out/$tag/tests.log"; exit 1; }
tail -3 "gpurun_out/$tag/tests.log"
LIBS="lib/libhrt_retire0.so lib/libhrt.so lib/libhrt_tailprio.so" bash scripts/ab_lib.sh "--steps 10" c2 2>&1 | tee "gpurun_out/$tag/ab.txt"
