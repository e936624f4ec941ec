#!/usr/bin/env bash
# Round-6 batch M: the C2 tail by dispatch order (wave index deciles: last job length, jobs taken, end time).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06m}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
python3 - "gpurun_out/$tag/wave_tail_c2.log" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
for k, v in d.items():
    print(k)
    for i, g in enumerate(v["by_dispatch_decile"]):
        print("  decile", i, g)
PY
