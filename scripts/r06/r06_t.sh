#!/usr/bin/env bash
# Round-6 batch T: rt_params.fold 3 (each launch folds the one before; auto with the automatic budget) — its tests, the
# timed compositions, the fold-related parity tests, then the default C3 / C5 bench lines against fold 1.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06t}"
mkdir -p "gpurun_out/$tag"
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/test_gpu_fold_next.py} \
  tests/test_gpu_timed.py "tests/test_gpu_parity.py::test_default_budget_launches_of_320_frames" \
  "tests/test_gpu_parity.py::test_fold_allocation_failure_shrinks_the_launches" \
  "tests/test_gpu_parity.py::test_fold_memory_follows_the_budget" \
  "tests/test_gpu_parity.py::test_release_scratch_then_draw_again" > "gpurun_out/$tag/tests.log" 2>&1 \
  || { tail -40 "gpurun_out/$tag/tests.log"; exit 1; }
tail -2 "gpurun_out/$tag/tests.log"
for round in 1 2; do
  for fold in 1 0; do
    timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 --fold $fold \
      > "gpurun_out/$tag/c3_fold$fold.log" 2>&1 || exit 1
    echo "c3 fold=$fold $(tail -1 gpurun_out/$tag/c3_fold$fold.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['config']['fold'], d['config']['fold_bytes'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
