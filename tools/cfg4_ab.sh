set -o pipefail
O=gpurun_out/r5c4
mkdir -p $O
timeout -k 10 120 tools/div_probe > $O/div_probe.json 2>&1 || exit 1
cat $O/div_probe.json
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_padding.py -m gpu -k "robust or trimmed or median or nan or special or pad or division" > $O/tests.log 2>&1 || { tail -20 $O/tests.log; exit 1; }
tail -2 $O/tests.log
bash tools/lib_ab.sh $O/ab tools/libp2pdl_prevq.so 3 cfg4-trimmed > $O/ab.txt 2>&1 || exit 1
cat $O/ab.txt
timeout -s KILL 220 rocprofv3 --kernel-trace --pmc SQ_WAVES SQ_INSTS_VALU SQ_ACTIVE_INST_VALU SQ_WAIT_INST_ANY SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_ANY SQ_WAIT_ANY GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $O/pmc_sq -o run -- python3 -u bench.py --no-sub --no-cpu-baseline --no-reference-gpu --steps 2 --warmup 1 --workload cfg4-trimmed > $O/pmc_sq.log 2>&1 || exit 1
python3 tools/rocpd_summary.py $O/pmc_sq robust > $O/sq_cfg4-trimmed.json
grep -h "valu_insts_per_wave" $O/sq_cfg4-trimmed.json
