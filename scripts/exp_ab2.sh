# A/B of two prebuilt libs ($A, $B) on configs $CFGS, after parity of $B
set -e
mkdir -p gpurun_out/ab
HRT_LIB=lib/$B timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x > gpurun_out/ab/pytest.log 2>&1 || { tail -30 gpurun_out/ab/pytest.log; exit 1; }
tail -1 gpurun_out/ab/pytest.log
for cfg in $CFGS; do
for lib in $A $B $A $B; do
  HRT_LIB=lib/$lib timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab/b.log 2>&1
  echo "$cfg $lib $(tail -1 gpurun_out/ab/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'])")"
done
done
