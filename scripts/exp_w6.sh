set -e
mkdir -p gpurun_out/exp5
for lib in libhrt.so libhrt_w6.so; do
  for cfg in c3 c4 c2; do
    HRT_LIB=lib/$lib timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp5/${lib}_$cfg.log 2>&1
    echo "$lib $cfg $(tail -1 gpurun_out/exp5/${lib}_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
