set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/kt_small
mkdir -p $O
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/a -o kt --output-format csv -- python3 $R/tools/span_pmc.py 3906250 3906314 > $O/log.txt 2>&1
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/b -o kt --output-format csv -- python3 $R/tools/span_pmc.py 7812500 7812564 >> $O/log.txt 2>&1
