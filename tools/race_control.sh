#!/bin/bash
# Negative control of tests/test_race_gpu.py: the race fixtures must PASS on
# the shipped library and FAIL on build_var/libgsr_lwrace.so, the round-5 batched per-entry sum
# update (commit 3ec9d20) rebuilt with -DGSR_BWD_LWPAR=1 by
#   tools/build_variants.sh lwrace "-DGSR_BWD_LWPAR=1"
# Usage (on the GPU box, repo root): bash tools/race_control.sh  -> gpurun_out/race_control.txt
set -o pipefail
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
out=gpurun_out/race_control.txt
run() {  # label, then the library path ("" = in-tree)
  echo "== $1" >> $out
  if [ -n "$2" ]; then export GSR_LIBRARY=$2; else unset GSR_LIBRARY; fi
  timeout -k 10 400 python3 -u -m pytest -q -rA -s --timeout 300 --timeout-method thread -m gpu tests/test_race_gpu.py \
    > gpurun_out/race_$3.txt 2>&1
  rc=$?
  grep -E "^\[(race3d|ties|close|grad)\]|^(PASSED|FAILED|ERROR)|passed|failed" gpurun_out/race_$3.txt >> $out
  echo "exit $rc" >> $out
  return $rc
}
: > $out
run "shipped library (pose-splatter_amd/gsr/lib/libgsr.so): must pass" "" head || exit 1
# a pytest failure is the expected outcome here; a crash / timeout (rc >= 124) is not
run "negative control build_var/libgsr_lwrace.so (GSR_BWD_LWPAR=1): must FAIL" "$PWD/build_var/libgsr_lwrace.so" lwrace
rc=$?
[ $rc -eq 1 ] && echo "negative control failed as required" >> $out && exit 0
echo "negative control did NOT fail (rc $rc)" >> $out
exit 1
