set -e
mkdir -p gpurun_out/q
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "variant or culling or zero_radius or rtiow or queue" > gpurun_out/q/pytest.log 2>&1 || { tail -30 gpurun_out/q/pytest.log; exit 1; }
tail -1 gpurun_out/q/pytest.log
for cfg in ${CFGS:-c3}; do
timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/q/b.log 2>&1
echo "$cfg $(tail -1 gpurun_out/q/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['box_tests_per_ray'], r['sphere_tests_per_ray'])")"
done
