set -e
mkdir -p gpurun_out/exp8
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "variant or culling or zero_radius or rtiow" > gpurun_out/exp8/pytest.log 2>&1 || { tail -30 gpurun_out/exp8/pytest.log; exit 1; }
tail -1 gpurun_out/exp8/pytest.log
for lib in libhrt_f0r0.so libhrt_f1r0.so libhrt_f0r1.so libhrt.so; do
  HRT_LIB=lib/$lib timeout -k 10 300 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/exp8/b.log 2>&1
  echo "$lib $(tail -1 gpurun_out/exp8/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['box_tests_per_ray'], r['sphere_tests_per_ray'])")"
done
