set -o pipefail
OUT=gpurun_out/labself; mkdir -p $OUT
export PYTHONUNBUFFERED=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
for lib in lab lab_noxor; do
 for r in median trimmed; do
  P2P_LIB=tools/libp2pdl_$lib.so timeout -k 10 300 python -u tools/lab_robust.py --rule $r --peers 256 --variants 0,6 > $OUT/${lib}_$r.log 2>&1 || { tail -20 $OUT/${lib}_$r.log; exit 1; }
  grep -h '^{' $OUT/${lib}_$r.log
 done
done
