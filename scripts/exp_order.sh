set -e
mkdir -p gpurun_out/exp7
timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -q -m gpu -x -k "queue or schedule or draw_frames" > gpurun_out/exp7/pytest.log 2>&1 || { tail -30 gpurun_out/exp7/pytest.log; exit 1; }
tail -1 gpurun_out/exp7/pytest.log
for cfg in c3 c4 c2; do
  for jf in 4 8; do
    timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --job-frames $jf > gpurun_out/exp7/b.log 2>&1
    echo "$cfg jf$jf $(tail -1 gpurun_out/exp7/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
timeout -k 10 200 env HRT_LIB=lib/libhrt_diag.so python scripts/stamps.py --config c4 --frames 64 --variants 1
