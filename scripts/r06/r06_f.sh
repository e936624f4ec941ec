#!/usr/bin/env bash
# Round-6 batch F: the C2 launch-end tail, rounds and shader cycles per round during each wave's last job (diagnostic
# build, scripts/wave_tail.py). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06f}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
python3 - "gpurun_out/$tag/wave_tail_c2.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(k, json.dumps({kk: vv for kk, vv in v.items() if kk not in ("resident_waves_timeline",)}))
PY
