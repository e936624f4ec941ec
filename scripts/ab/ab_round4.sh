set -u
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/ab1
for round in 1 2; do
 for cfg in c3 c4 c5; do
  extra=""; [ $cfg = c5 ] && extra="--frames 256"
  for lib in lib/libhrt.so lib/libhrt_noslp.so lib/libhrt_leafiv.so lib/libhrt_both.so; do
    tag=$(basename $lib .so)
    HRT_LIB=$lib timeout -k 10 200 python bench.py --config $cfg --steps 3 --warmup 1 --emulate-ranks 0 --no-cpu-baseline --no-golden $extra > gpurun_out/ab1/${cfg}_${tag}_$round.log 2>&1
    rc=$?
    echo "$round $cfg $tag rc=$rc $(tail -1 gpurun_out/ab1/${cfg}_${tag}_$round.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])" 2>/dev/null)"
    case $rc in 0) ;; *) echo stop; exit $rc;; esac
  done
 done
done
