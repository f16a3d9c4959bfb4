#!/bin/bash
# Run GPU steps in order, each under its own time limit; stop at the first
# fault-like exit (timeout 124/137, abort 134, segfault 139, any signal > 128).
# Ordinary failures (exit 1/2, e.g. a failing test) are logged and the run goes on.
#   tools/gpu_steps.sh "name|seconds|command" ...
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in "$@"; do
  name="${spec%%|*}"; rest="${spec#*|}"; secs="${rest%%|*}"; cmd="${rest#*|}"
  echo "=== [$name] (limit ${secs}s): $cmd"
  start=$(date +%s)
  timeout -k 10 "$secs" bash -c "$cmd" > "gpurun_out/$name.log" 2>&1
  rc=$?
  echo "=== [$name] rc=$rc in $(( $(date +%s) - start ))s"
  tail -n 25 "gpurun_out/$name.log"
  if [ $rc -ge 124 ]; then
    echo "=== stopping: fault-like exit $rc"
    exit $rc
  fi
done
