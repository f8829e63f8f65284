#!/bin/bash
# Round 6 (last session): the default bench line with cfg2's general path
# also timed over the slab rows' own views (same route, one allocation).
set -o pipefail
O=gpurun_out/bench_views
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT" || exit 1
export PYTHONUNBUFFERED=1
timeout -k 10 600 python3 -u bench.py > $O/bench.json 2> $O/bench.err || { tail -30 $O/bench.err; exit 1; }
python3 -c "
import json
d=json.loads(open('$O/bench.json').readline())
print('main', d['value'], d['roofline']['frac'])
print(json.dumps(d['sub']['cfg2_dropin'].get('general_path'), indent=1))
"
