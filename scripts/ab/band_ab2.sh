#!/usr/bin/env bash
# (Historical: the pipelined band launches this measured were removed after these A/Bs (commit 512dacf); the
# results are in profiles/r04/band/. The lines' config no longer carries a 'bands' field.)
# Bands with one side stream (sequential band traces; folds beside them) vs two, at 8 GiB, against one launch;
# then the suspend_below re-tune (scripts/sweep_r4.sh).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bandab2
for round in 1 2; do
  for cfg in c3 c4; do
    for v in "lib/libhrt.so:32768" "lib/libhrt.so:8192" "lib/libhrt_s1.so:8192"; do
      lib=${v%%:*}; mb=${v#*:}; tag=$(basename $lib .so)_$mb
      HRT_LIB=$lib timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --emulate-ranks 0 --no-cpu-baseline \
        --no-golden --queue-budget-mb $mb > gpurun_out/bandab2/${cfg}_${tag}_$round.log 2>&1 || exit $?
      echo "$round $cfg $tag $(tail -1 gpurun_out/bandab2/${cfg}_${tag}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['config']['bands'])")"
    done
  done
done
bash scripts/sweep_r4.sh
