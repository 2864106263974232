"""The A/B-selectable encoder variants stay bit-exact.

The library picks one kernel per job shape and reads its A/B knobs once per
process, so the non-default forms are only reachable from a fresh process:
  * (round 3's CDA_RS16_HALF=0 full-width GF(2^16) kernel was removed in round 4
    with the byte-form encoders it belonged to; the bitsliced encoder has no
    variants)
  * CDA_RS8_SLICE=0 -- the k = 128 Q0 launch of a batch without the XCD-aware
    128-byte slices (mode 0, two codewords per workgroup);
  * CDA_RS8_BS=1 -- round 1's four-codeword k = 128 encoder.
Each child extends squares of the committed fixtures and compares data roots
and EDS / root digests (tests/golden/k512.json, config4_k128.json; generated
by oracle/gen_config4.py from the C oracle).  Reference: the Leopard encoders
behind pkg/appconsts/global_consts.go:92 (klauspost/reedsolomon v1.12.1)."""
import json
import os
import subprocess
import sys

import pytest

import knobs

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)

_CHILD = r"""
import hashlib, json, os, sys
sys.path[:0] = [os.path.join(ROOT, "celestia-app_amd"), ROOT]
import numpy as np
import torch
from celestia_da import Context, testfactory
mode, k, n = sys.argv[1], int(sys.argv[2]), int(sys.argv[3])
W = 2 * k
ctx = Context(0)
dev = torch.device("cuda", 0)
eds = torch.zeros(n, W * W * 512, dtype=torch.uint8, device=dev)
for i in range(n):
    eds[i].view(W, W, 512)[:k, :k] = torch.from_numpy(testfactory.random_square(k, i)).to(dev).view(k, k, 512)
rows = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
cols = torch.empty(n, W * 90, dtype=torch.uint8, device=dev)
roots = torch.empty(n, 32, dtype=torch.uint8, device=dev)
status = torch.empty(n, dtype=torch.int32, device=dev)
ctx.extend_dah_inplace_device(k, n, eds.data_ptr(), rows.data_ptr(), cols.data_ptr(), roots.data_ptr(),
                              status.data_ptr(), torch.cuda.current_stream(dev).cuda_stream)
torch.cuda.synchronize()
sha = lambda t: hashlib.sha256(t.cpu().numpy().tobytes()).hexdigest()
out = [{"status": int(status[i]), "data_root": roots[i].cpu().numpy().tobytes().hex(),
        "eds_sha256": sha(eds[i]), "row_roots_sha256": sha(rows[i]), "col_roots_sha256": sha(cols[i])}
       for i in range(n)]
print(json.dumps(out))
""".replace("ROOT", repr(ROOT))


def _run(env_extra: dict, k: int, n: int) -> list:
    env = dict(os.environ)
    env.update(env_extra)
    env["CDA_LIB"] = knobs.lib_path_for_tests()   # the A/B knobs are read only by the test build
    r = subprocess.run([sys.executable, "-c", _CHILD, "x", str(k), str(n)], env=env, capture_output=True,
                       text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    return json.loads(r.stdout.strip().splitlines()[-1])


@pytest.mark.parametrize("env", [{"CDA_RS8_SLICE": "0"}, {"CDA_RS8_SLICE": "1"}, {"CDA_RS8_BS": "1"}],
                         ids=["mode0", "slices", "round1_kernel"])
def test_gf8_q0_modes_match_fixture(env):
    """16 squares in one submission (the batch path: slice mode 2 unless
    CDA_RS8_SLICE=0; CDA_RS8_BS=1 is round 1's four-codeword kernel) against
    config 4's fixture (squares 0..15)."""
    g = json.load(open(os.path.join(HERE, "golden", "config4_k128.json")))["squares"]
    got = _run(env, 128, 16)
    for i in range(16):
        want = g[str(i)]
        assert got[i]["status"] == 0
        assert got[i]["data_root"] == want["data_root"], i
        assert got[i]["row_roots_sha256"] == want["row_roots_sha256"], i
        assert got[i]["col_roots_sha256"] == want["col_roots_sha256"], i
        if "eds_sha256" in want:
            assert got[i]["eds_sha256"] == want["eds_sha256"], i
