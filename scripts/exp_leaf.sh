set -e
mkdir -p gpurun_out/exp6
run() {
  timeout -k 10 300 env "$@" python bench.py --config c3 --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/exp6/b.log 2>&1
  echo "$* $(tail -1 gpurun_out/exp6/b.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print(d['value'], d['ms_per_step'], r['box_tests_per_ray'], r['sphere_tests_per_ray'])")"
}
run HRT_BVH_MAX_LEAF=3 HRT_BVH_LEAF_DEPTH=0
run HRT_BVH_MAX_LEAF=5 HRT_BVH_LEAF_DEPTH=0
run HRT_BVH_MAX_LEAF=6 HRT_BVH_LEAF_DEPTH=0
run HRT_BVH_MAX_LEAF=8 HRT_BVH_LEAF_DEPTH=99 HRT_BVH_TRAVERSAL_COST=1
run HRT_BVH_MAX_LEAF=8 HRT_BVH_LEAF_DEPTH=99 HRT_BVH_TRAVERSAL_COST=2
run HRT_BVH_MAX_LEAF=8 HRT_BVH_LEAF_DEPTH=99 HRT_BVH_TRAVERSAL_COST=4
