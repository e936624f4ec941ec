#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Pipelined bands vs one launch: the band GPU tests, kernel-trace timelines, and interleaved bench A/B on C3/C4/C5
# (C5 at 1024 spp) with the 8 GiB budget against 32 GiB (one launch for C3 / C4).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bandab
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "band_pipeline or ranks_beyond or fold_allocation or fold_memory" > gpurun_out/bandab/tests.log 2>&1 || { tail -30 gpurun_out/bandab/tests.log; exit 1; }
tail -2 gpurun_out/bandab/tests.log
bash scripts/band_trace.sh 8192 b8g || exit $?
for round in 1 2; do
  for cfg in c3 c4 c5; do
    extra=""; [ $cfg = c5 ] && extra="--frames 1024"
    for mb in 32768 8192; do
      timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
        --queue-budget-mb $mb $extra > gpurun_out/bandab/${cfg}_${mb}_$round.log 2>&1 || exit $?
      echo "$round $cfg $mb $(tail -1 gpurun_out/bandab/${cfg}_${mb}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['fold_bytes'])")"
    done
  done
done
