#!/usr/bin/env bash
# Round-6 batch O: the C2 tail with the single job counter (HRT_NQ=0: lib/libhrt_diag_nq0.so, lib/libhrt_nq0.so) against
# the per-XCD queues — wave records, then a same-box A/B with the 8-way emulated split.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06o}"
mkdir -p "gpurun_out/$tag"
for lib in lib/libhrt_diag.so lib/libhrt_diag_nq0.so; do
  n=$(basename $lib .so)
  HRT_LIB=$lib timeout -k 10 120 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
    > "gpurun_out/$tag/wave_tail_c2_$n.log" 2>&1 || exit 1
  python3 - "gpurun_out/$tag/wave_tail_c2_$n.log" $n <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(sys.argv[2], k, json.dumps({kk: v[kk] for kk in ("trace_ms", "tail_after_first_drain_ms", "drain_ms_pcts", "last_job_to_end_ms_pcts")}),
          json.dumps(v["jobs"]["last_5pct_takes"]))
PY
done
LIBS="lib/libhrt.so lib/libhrt_nq0.so" bash scripts/ab_lib.sh "--steps 10" c2 2>&1 | tee "gpurun_out/$tag/ab.txt"
