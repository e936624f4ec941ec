# BVH4 check: parity tests for the new variants, then the C3 bench per variant.
set -e
mkdir -p gpurun_out/exp2
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -k "variant or culling or zero_radius" > gpurun_out/exp2/pytest.log 2>&1 || { tail -30 gpurun_out/exp2/pytest.log; exit 1; }
tail -2 gpurun_out/exp2/pytest.log
for v in 4 9 10; do
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --frames-per-launch 1024 --variant $v > gpurun_out/exp2/bench_v$v.log 2>&1
  echo "v$v $(tail -1 gpurun_out/exp2/bench_v$v.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['box_tests_per_ray'], d['roofline']['sphere_tests_per_ray'])")"
done
