set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/span_pmc
mkdir -p $O
for cfg in "15625000 15625064" "15625000 125000000"; do
  set -- $cfg
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_UTCL1_THRASHING_STALL_sum -d $O/p$2 -o pmc --output-format csv -- python3 $R/tools/span_pmc.py $1 $2 > $O/log_$2.txt 2>&1
  timeout -s KILL 120 rocprofv3 --pmc TCP_UTCL1_STALL_UTCL2_REQ_OUT_OF_CREDITS_sum TCP_UTCL1_SERIALIZATION_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum -d $O/q$2 -o pmc --output-format csv -- python3 $R/tools/span_pmc.py $1 $2 >> $O/log_$2.txt 2>&1
done
