# A/B: default lib vs $ALT (HRT_LIB), C3, after parity of the alternative
set -e
mkdir -p gpurun_out/ab
HRT_LIB=lib/$ALT timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "variant or culling or zero_radius or rtiow or queue" > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for lib in libhrt.so $ALT libhrt.so $ALT; do
  HRT_LIB=lib/$lib timeout -k 10 300 python bench.py --config ${CFG:-c3} --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab/b.log 2>&1
  echo "$lib $(tail -1 gpurun_out/ab/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['box_tests_per_ray'], r['sphere_tests_per_ray'])")"
done
