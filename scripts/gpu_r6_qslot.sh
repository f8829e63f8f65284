#!/bin/bash
# Round 6 (late): captured split launches keep a reserved tile-queue pair.
# The new concurrency test on the product build, the whole GPU suite, then
# the same test against the previous build (captured launches on a rotating
# pair): informational, an assertion failure there is the finding.
set -o pipefail
O=gpurun_out/qslot3
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
step() {  # step <seconds> <log> <cmd...>
  local secs=$1 logf=$2; shift 2
  echo "== $(date +%T) $*" | tee -a $O/steps.log
  timeout -k 10 "$secs" "$@" > "$logf" 2>&1
  local rc=$?
  echo "== rc=$rc" | tee -a $O/steps.log
  tail -4 "$logf"
  return $rc
}
step 240 $O/new_test.log python3 -u -m pytest tests/test_gpu_graph.py -m gpu -x -v -s --timeout 150 \
  --timeout-method thread -k captured_split || exit $?
[ -n "$FULL" ] && { step 500 $O/pytest.log python3 -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread || exit $?; }
P2P_LIB=$PWD/tools/libp2pdl_old.so step 240 $O/old_lib.log python3 -u -m pytest tests/test_gpu_graph.py -m gpu \
  -x -v -s --timeout 150 --timeout-method thread -k captured_split
rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
exit 0
