# Round 6 t: cfg2 drop-in line x3 (the general path's per-call spread).
set -o pipefail
O=gpurun_out/r06t; mkdir -p $O
for i in 1 2 3; do
  timeout -k 10 300 python -u bench.py --workload cfg2-dropin --no-cpu-baseline --no-reference-gpu > $O/cfg2_$i.json 2> $O/cfg2_$i.err || { tail $O/cfg2_$i.err; exit 1; }
  python -c "import json; d=json.loads(open('$O/cfg2_$i.json').readline()); g=d['general_path']; print(d['ms_per_step'], g['us_per_call'], g['kernel_ms'], g['us_per_call_new_table_every_call'])"
done
echo done
