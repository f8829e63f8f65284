#!/bin/bash
# product GPU tests, then the persistent-pair lab library's multi-tile probe
set -o pipefail
OUT=gpurun_out/chk; mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
P2P_LIB=tools/libp2pdl_persist.so bash tools/hang_probe.sh "median nonan 32768" "median nonan 32832" "median nonan 40000"
