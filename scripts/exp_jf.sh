set -e
mkdir -p gpurun_out/exp4
export TMPDIR=/tmp
for jf in 8 32 64; do
  timeout -k 10 300 python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --job-frames $jf > gpurun_out/exp4/bench_c3_j$jf.log 2>&1
  echo "c3 jf$jf $(tail -1 gpurun_out/exp4/bench_c3_j$jf.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['ms_per_step'])")"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/exp4/prof -o run --output-format csv -- python3 bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline --job-frames 16 > gpurun_out/exp4/prof.log 2>&1
find gpurun_out/exp4/prof -name "*kernel_stats.csv" | head -1 | xargs cat
