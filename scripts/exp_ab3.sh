# A/B of two prebuilt libs ($A, $B) with bench args $ARGS (no parity step)
set -e
mkdir -p gpurun_out/ab
for lib in $A $B $A $B; do
  HRT_LIB=lib/$lib timeout -k 10 300 python bench.py $ARGS --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/b.log 2>&1
  echo "$lib $(tail -1 gpurun_out/ab/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['kernel'])")"
done
