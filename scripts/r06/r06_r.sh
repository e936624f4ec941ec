#!/usr/bin/env bash
# Round-6 batch R: each launch folds the one before inside its own waves (HRT_FOLD_NEXT = fold_mod, the fraction of
# waves that fold first; unset = k_accumulate after every launch). The C3 timed composition against the oracle with
# folding on, then a same-box A/B of fold_mod on C3.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06r}"
mkdir -p "gpurun_out/$tag"
[ -n "${SKIP_TESTS:-}" ] || HRT_FOLD_NEXT=8 timeout -k 10 300 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu \
  "tests/test_gpu_timed.py::test_c3_as_timed_crosses_the_ema_switch_inside_a_launch" > "gpurun_out/$tag/tests.log" 2>&1 \
  || { tail -30 "gpurun_out/$tag/tests.log"; exit 1; }
tail -2 "gpurun_out/$tag/tests.log"
for round in 1 2; do
  for fm in ${FMS:-0 8 4 16 1}; do
    if [ "$fm" = 0 ]; then unset HRT_FOLD_NEXT; else export HRT_FOLD_NEXT=$fm; fi
    timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_f$fm.log" 2>&1 || exit 1
    echo "c3 fold_mod=$fm $(tail -1 gpurun_out/$tag/c3_f$fm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['config']['fold_bytes'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
