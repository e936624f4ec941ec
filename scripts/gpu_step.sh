#!/usr/bin/env bash
# Run GPU steps in order, each under its own time limit; stop at the first crash-like exit
# (timeout 124/137, abort 134, segfault 139). Ordinary test failures (exit 1) do not stop later steps.
# usage: scripts/gpu_step.sh "<name>" <seconds> <command...> [--- "<name>" <seconds> <command...>]...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
while [ $# -gt 0 ]; do
  name="$1"; secs="$2"; shift 2
  cmd=()
  while [ $# -gt 0 ] && [ "$1" != "---" ]; do cmd+=("$1"); shift; done
  [ $# -gt 0 ] && shift
  echo "=== $name (limit ${secs}s): ${cmd[*]}"
  start=$(date +%s)
  timeout -k 10 "$secs" "${cmd[@]}" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== $name exit $rc after $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  case $rc in
    0|1|2|5) ;;
    *) echo "=== stopping: crash-like exit $rc"; exit $rc ;;
  esac
done
