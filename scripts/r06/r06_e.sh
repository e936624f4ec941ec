#!/usr/bin/env bash
# Round-6 batch E: (1) the C2 launch-end tail — wave records of the diagnostic build (8-word records: shader clock at
# start / drain / end, lanes in flight at the drain, samples finished after the last job take, rounds after the drain)
# for ranks 0 and 4 of 8 and the full image; (2) C4's HBM bytes per launch — the learning launch (warmup 0, as the
# round-5 PMC passes ran) against the timed, cost-ordered launch (warmup 1, last dispatch) and raster order (cost_order
# 1). Logs: gpurun_out/<tag>/.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
tag="${1:-r06e}"
mkdir -p "gpurun_out/$tag"
HRT_LIB=lib/libhrt_diag.so timeout -k 10 300 python scripts/wave_tail.py --config c2 --ranks 8 --rank 0 4 --full \
  > "gpurun_out/$tag/wave_tail_c2.log" 2>&1 || exit 1
tail -c 4000 "gpurun_out/$tag/wave_tail_c2.log"
for v in "learn 0 0" "ordered 1 0" "raster 1 1"; do
  set -- $v
  name=$1; warm=$2; co=$3
  d="gpurun_out/$tag/c4_$name"
  mkdir -p "$d"
  extra=""
  [ "$co" = 1 ] && extra="--cost-order 1"
  i=0
  for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
    i=$((i+1))
    timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$d" -o "p$i" -- python3 bench.py --config c4 \
      --no-cpu-baseline --no-golden --steps 1 --warmup $warm $extra > "$d/p$i.log" 2>&1 || exit 1
  done
  PMC_DISPATCH=last python3 scripts/pmc_summary.py "$d" > /dev/null || exit 1
  python3 -c "import json; s=json.load(open('$d/pmc_summary.json')); print('$name', round(s['hbm_read_bytes_per_launch']/1e9,3), round(s['hbm_write_bytes_per_launch']/1e9,3), round(s['TCC_HIT_sum']/(s['TCC_HIT_sum']+s['TCC_MISS_sum']),4), s['_dispatches_per_pass'])" | tee -a "gpurun_out/$tag/c4_pmc.txt"
done
