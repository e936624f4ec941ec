#!/usr/bin/env bash
# Round-6 batch S: in-launch fold of the previous launch (HRT_FOLD_NEXT = fold_mod) on the mixed kernel too: the C5 timed
# composition against the oracle with folding on, a fold_mod sweep on C3, and C5 with / without.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
tag="${1:-r06s}"
mkdir -p "gpurun_out/$tag"
HRT_FOLD_NEXT=16 timeout -k 10 400 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu \
  "tests/test_gpu_timed.py::test_c5_as_timed_in_twelve_launches" > "gpurun_out/$tag/tests.log" 2>&1 \
  || { tail -30 "gpurun_out/$tag/tests.log"; exit 1; }
tail -2 "gpurun_out/$tag/tests.log"
for round in 1 2; do
  for fm in 0 16 32 64 128; do
    if [ "$fm" = 0 ]; then unset HRT_FOLD_NEXT; else export HRT_FOLD_NEXT=$fm; fi
    timeout -k 10 300 python bench.py --config c3 --no-cpu-baseline --no-golden --steps 5 --emulate-ranks 0 \
      > "gpurun_out/$tag/c3_f$fm.log" 2>&1 || exit 1
    echo "c3 fold_mod=$fm $(tail -1 gpurun_out/$tag/c3_f$fm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['achieved'], d['config']['fold_bytes'])")"
  done
done | tee "gpurun_out/$tag/ab_c3.txt"
for fm in 0 16; do
  if [ "$fm" = 0 ]; then unset HRT_FOLD_NEXT; else export HRT_FOLD_NEXT=$fm; fi
  timeout -k 10 300 python bench.py --config c5 --no-cpu-baseline --no-golden --steps 1 --warmup 1 --emulate-ranks 0 \
    > "gpurun_out/$tag/c5_f$fm.log" 2>&1 || exit 1
  echo "c5 fold_mod=$fm $(tail -1 gpurun_out/$tag/c5_f$fm.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done | tee "gpurun_out/$tag/ab_c5.txt"
