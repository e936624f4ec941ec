#!/usr/bin/env bash
# (The rt_params.pipeline build it measured was removed after this batch: DESIGN.md §6 Round 6.)
# Round-6 batch P: pipelined launches (rt_params.pipeline) — the pipeline tests and the timed compositions that now run
# pipelined, then a same-box A/B of pipeline 1 (off) against the default (auto = on) on C3 and C5.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06p}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_gpu_pipeline.py \
  "tests/test_gpu_timed.py::test_c3_as_timed_crosses_the_ema_switch_inside_a_launch" \
  "tests/test_gpu_parity.py::test_default_budget_launches_of_320_frames" \
  "tests/test_gpu_parity.py::test_fold_allocation_failure_shrinks_the_launches" > "gpurun_out/$tag/tests.log" 2>&1 || { tail -30 "gpurun_out/$tag/tests.log"; exit 1; }
tail -3 "gpurun_out/$tag/tests.log"
for round in 1 2; do
  for pl in 1 0; do
    timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 --pipeline $pl \
      > "gpurun_out/$tag/c3_p$pl.log" 2>&1 || exit 1
    echo "c3 pipeline=$pl $(tail -1 gpurun_out/$tag/c3_p$pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('pipelined'), d['roofline']['achieved'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
for pl in 1 0; do
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 --pipeline $pl \
    > "gpurun_out/$tag/c5_p$pl.log" 2>&1 || exit 1
  echo "c5 pipeline=$pl $(tail -1 gpurun_out/$tag/c5_p$pl.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config'].get('pipelined'))")"
done | tee "gpurun_out/$tag/ab_c5.txt"
