set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r3d
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r3d/gputest.log 2>&1 || exit 1
run() {  # name args
  timeout -k 10 400 python -u bench.py --no-cpu-baseline --no-golden $2 > gpurun_out/r3d/$1.log 2>&1 || return 1
  echo "$1 $(tail -1 gpurun_out/r3d/$1.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); e=d.get('emulated_split') or {}; print(d['value'], d['ms_per_step'], d['roofline']['kernel'], e.get('efficiency'), e.get('predicted_ms_per_step'))")"
}
for round in 1 2; do
  run c3_steal_$round "--config c3 --steps 3 --emulate-ranks 8" || exit 1
  run c3_nosteal_$round "--config c3 --steps 3 --emulate-ranks 8 --steal 1" || exit 1
  run c4_steal_$round "--config c4 --steps 3 --emulate-ranks 8" || exit 1
  run c4_nosteal_$round "--config c4 --steps 3 --emulate-ranks 8 --steal 1" || exit 1
  run c5_steal_$round "--config c5 --frames 256 --steps 2 --emulate-ranks 0" || exit 1
  run c5_nosteal_$round "--config c5 --frames 256 --steps 2 --emulate-ranks 0 --steal 1" || exit 1
done
