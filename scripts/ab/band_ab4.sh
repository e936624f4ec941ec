#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Drain-fold bands (four buffers; band i folds band i - 2 in its drain): parity tests, then 8 GiB bands against one
# launch (32 GiB) on C3 / C4 / C5 (C4 also with stealing forced on for the band launches).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bandab4
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_parity.py \
  -k "band_pipeline or fold or accumulate" > gpurun_out/bandab4/pytest.log 2>&1 || { tail -30 gpurun_out/bandab4/pytest.log; exit 1; }
tail -3 gpurun_out/bandab4/pytest.log
run() {  # cfg mb steal tag steps
  timeout -k 10 300 python bench.py --config $1 --steps $5 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden \
    --queue-budget-mb $2 --steal $3 > gpurun_out/bandab4/$1_$2_s$3_$4.log 2>&1 || return $?
  echo "$4 $1 $2 steal=$3 $(tail -1 gpurun_out/bandab4/$1_$2_s$3_$4.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['bands'])")"
}
for round in 1 2; do
  run c3 32768 0 $round 3 && run c3 8192 0 $round 3 || exit 1
done
for round in 1 2; do
  run c4 32768 0 $round 2 && run c4 8192 0 $round 2 && run c4 8192 2 $round 2 || exit 1
done
run c5 32768 0 1 1 && run c5 8192 0 1 1 || exit 1
