"""GF(2^16) one-launch extension (rs_gf16_bs.hip rs16_bs_ticket_kernel): Q0
rows + columns and Q3 of a batch in ONE ticketed launch, the Q3 workgroups
reading Q2 parity that other workgroups of the same launch wrote (write-through
stores, agent-scope acquire).  Checked against the two-launch path
(CDA_RS16_TICKET=0) in two contexts and the oracle, under uneven load (a
matrix-multiply stream beside it) with the EDS arena pre-filled with a poison
pattern before every call, so a stale Q2 read shows as wrong Q3 bytes."""
import os

import numpy as np
import pytest

import coracle
from celestia_da import Context

pytestmark = pytest.mark.gpu


def _context(ticket):
    old = os.environ.get("CDA_RS16_TICKET")
    os.environ["CDA_RS16_TICKET"] = "1" if ticket else "0"
    try:
        return Context(0)
    finally:
        if old is None:
            del os.environ["CDA_RS16_TICKET"]
        else:
            os.environ["CDA_RS16_TICKET"] = old


@pytest.mark.parametrize("k,n,reps", [(256, 6, 8), (512, 2, 4)])
def test_ticket_launch_matches_two_launches_under_load(k, n, reps):
    import torch
    dev = torch.device("cuda", 0)
    W = 2 * k
    ods = np.stack([coracle.random_square(k, 300 + i) for i in range(n)])
    d_ods = torch.from_numpy(ods.reshape(n, -1)).to(dev)

    def outs():
        return (torch.empty(n, W * W * 512, dtype=torch.uint8, device=dev),
                torch.empty(n, W * 90, dtype=torch.uint8, device=dev),
                torch.empty(n, W * 90, dtype=torch.uint8, device=dev),
                torch.empty(n, 32, dtype=torch.uint8, device=dev),
                torch.empty(n, dtype=torch.int32, device=dev))

    s = torch.cuda.current_stream(dev)
    ref_ctx, ctx = _context(False), _context(True)
    want = outs()
    ref_ctx.extend_dah_device(d_ods.data_ptr(), k, n, *[t.data_ptr() for t in want], s.cuda_stream)
    torch.cuda.synchronize()
    # the two-launch path against the oracle on the last square
    e_eds, _, _, e_root = coracle.cpu_baseline(ods[-1], 16)
    assert np.array_equal(want[0][-1].cpu().numpy().reshape(-1, 512), e_eds)
    assert want[3][-1].cpu().numpy().tobytes() == e_root

    load = torch.cuda.Stream(dev)
    a = torch.randn(4096, 4096, device=dev, dtype=torch.bfloat16)
    got = outs()
    for r in range(reps):
        with torch.cuda.stream(load):   # uneven load: matrix multiplies beside the launch
            for _ in range(3 + r % 3):
                a = (a @ a).clamp_(-1, 1)
        got[0].fill_(0xA5 ^ r)           # poison: a stale Q2 line would surface in Q3
        ctx.extend_dah_device(d_ods.data_ptr(), k, n, *[t.data_ptr() for t in got], s.cuda_stream)
        torch.cuda.synchronize()
        for x, y in zip(want, got):
            assert torch.equal(x, y), f"rep {r}"
