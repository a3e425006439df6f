#!/bin/bash
# Run GPU steps with per-step time limits; stop at the first crash/timeout
# (exit codes other than 0 / 1 = test failures), never retry.
mkdir -p gpurun_out
step() {
  local limit=$1; shift
  local name=$1; shift
  echo "=== $name ($(date +%T))"
  timeout -k 10 "$limit" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc ($(date +%T))"
  tail -5 "gpurun_out/$name.log"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  return 0
}
