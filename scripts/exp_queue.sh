# Sample-queue schedule: parity suite (default schedule = queue), then C3/C4 bench per schedule.
set -e
mkdir -p gpurun_out/exp3
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu > gpurun_out/exp3/pytest.log 2>&1 || { tail -40 gpurun_out/exp3/pytest.log; exit 1; }
tail -2 gpurun_out/exp3/pytest.log
for cfg in c3 c4; do
  for jf in 1 4 16; do
    timeout -k 10 300 python bench.py --config $cfg --steps 2 --warmup 1 --no-cpu-baseline --schedule 2 --job-frames $jf > gpurun_out/exp3/bench_${cfg}_j$jf.log 2>&1
    echo "$cfg jf$jf $(tail -1 gpurun_out/exp3/bench_${cfg}_j$jf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
  done
done
