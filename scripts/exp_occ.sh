set -e
mkdir -p gpurun_out/exp1
for lib in libhrt.so libhrt_s16.so libhrt_s16w8.so; do
  for fpl in 32 1024; do
    echo "== $lib fpl=$fpl"
    HRT_LIB=lib/$lib timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --frames-per-launch $fpl --variant 4 > gpurun_out/exp1/${lib}_$fpl.log 2>&1
    tail -1 gpurun_out/exp1/${lib}_$fpl.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])"
  done
done
