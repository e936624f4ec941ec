# Every BASELINE.json config on one GPU (C5 = its single-GPU share is the whole image here).
set -e
mkdir -p gpurun_out/all
for cfg in c1 c2 c3 c4; do
  timeout -k 10 600 python bench.py --config $cfg > gpurun_out/all/bench_$cfg.log 2>&1
  echo "$cfg $(tail -1 gpurun_out/all/bench_$cfg.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['achieved'], (d['roofline'].get('pmc') or {}).get('active_lanes'), d.get('cpu_baseline',{}).get('value'))")"
done
timeout -k 10 900 python bench.py --config c5 --steps 1 --warmup 1 > gpurun_out/all/bench_c5.log 2>&1
echo "c5 $(tail -1 gpurun_out/all/bench_c5.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['achieved'], (d['roofline'].get('pmc') or {}).get('active_lanes'), d.get('cpu_baseline',{}).get('value'))")"
