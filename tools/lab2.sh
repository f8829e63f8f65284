set -o pipefail
OUT=gpurun_out/r02c; mkdir -p $OUT
export PYTHONUNBUFFERED=1
timeout -k 10 300 python -u tools/lab_robust.py --rule median --peers 256 --variants 0,5 > $OUT/lab_med.log 2>&1 || { tail $OUT/lab_med.log; exit 1; }
timeout -k 10 300 python -u tools/lab_robust.py --rule trimmed --peers 256 --variants 0,5 > $OUT/lab_trim.log 2>&1 || { tail $OUT/lab_trim.log; exit 1; }
timeout -k 10 300 python -u tools/lab_robust.py --rule median --peers 200 --variants 0,5 --coords 20000000 > $OUT/lab_med200.log 2>&1 || { tail $OUT/lab_med200.log; exit 1; }
timeout -k 10 300 python -u tools/lab_robust.py --rule trimmed --peers 200 --variants 0,5 --coords 20000000 > $OUT/lab_trim200.log 2>&1 || { tail $OUT/lab_trim200.log; exit 1; }
grep -h '^{' $OUT/*.log
