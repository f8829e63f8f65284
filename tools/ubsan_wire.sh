#!/bin/bash
# Host-only sanitizer pass over the receive-path parser (csrc/wire.cpp): an
# UndefinedBehaviorSanitizer build of the CPython extension (no preload
# needed, unlike ASan), loaded in place of p2pdl_amd._wire for the CPU parser
# tests and a 20k-case corruption fuzz.  No GPU.
set -euo pipefail
OUT=${1:-/tmp/p2p_ubsan}
mkdir -p "$OUT"
ROOT=$(cd "$(dirname "$0")/.." && pwd)
PY_INC=$(python3 -c "import sysconfig; print(sysconfig.get_paths()['include'])")
g++ -O1 -g -std=c++17 -fPIC -shared -fsanitize=undefined -fno-sanitize-recover=undefined \
    -fno-omit-frame-pointer -I"$PY_INC" -o "$OUT/_wire.so" "$ROOT/p2pdl_amd/csrc/wire.cpp"
python3 - "$ROOT" "$OUT/_wire.so" <<'PY'
import importlib.util, pickle, sys
root, so = sys.argv[1], sys.argv[2]
sys.path.insert(0, root)
spec = importlib.util.spec_from_file_location("p2pdl_amd._wire", so)
mod = importlib.util.module_from_spec(spec)
spec.loader.exec_module(mod)
sys.modules["p2pdl_amd._wire"] = mod
import p2pdl_amd
p2pdl_amd._wire = mod
from p2pdl_amd.node import inbox
assert inbox._wire is mod
import numpy as np, pytest, torch
rc = pytest.main(["-q", "-x", f"{root}/tests/test_inbox.py", "-m", "not gpu", "-p", "no:cacheprovider"])
if rc:
    sys.exit(rc)
rng = np.random.default_rng(11)
sd = torch.nn.Sequential(torch.nn.Linear(30, 20), torch.nn.BatchNorm1d(20), torch.nn.Linear(20, 5)).state_dict()
base = [pickle.dumps(sd, protocol=p) for p in (3, 4, 5)]
ok = bad = 0
for it in range(20000):
    d = bytearray(base[it % 3])
    for i in rng.integers(0, len(d), int(rng.integers(1, 12))):
        d[i] = int(rng.integers(0, 256))
    if it % 7 == 0:
        d = d[:int(rng.integers(1, len(d)))]
    try:
        inbox.ZeroCopyParser(bytes(d), native=True).parse()
        ok += 1
    except pickle.UnpicklingError:
        bad += 1
print(f"ubsan fuzz: {ok} parsed, {bad} rejected, no undefined behaviour")
PY
