#!/usr/bin/env bash
# Round-6 batch I: the C2 launch-end tail with the sample stores dropped (lib/libhrt_diag_nostore.so) or the exit-time
# counter flush dropped (lib/libhrt_diag_noflush.so), timing-only diagnostic builds, against the diagnostic build.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06i}"
mkdir -p "gpurun_out/$tag"
for lib in lib/libhrt_diag.so lib/libhrt_diag_nostore.so lib/libhrt_diag_noflush.so; do
  n=$(basename $lib .so)
  HRT_LIB=$lib timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
    > "gpurun_out/$tag/wave_tail_c2_$n.log" 2>&1 || exit 1
  python3 - "gpurun_out/$tag/wave_tail_c2_$n.log" $n <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(sys.argv[2], k, json.dumps({kk: v[kk] for kk in ("trace_ms", "tail_after_first_drain_ms", "last_job_to_end_ms_pcts", "clk_per_round_last_job_pcts")}),
          json.dumps(v["jobs"]["last_5pct_takes"]))
PY
done
