"""k=512 single square: in-place vs packed entry, alternating blocks of calls
in one process (does the layout or the call order set the time?)."""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "celestia-app_amd"))
from celestia_da import Context, testfactory  # noqa: E402

k = 512
W = 2 * k
ctx = Context(0)
dev = torch.device("cuda", 0)
s = torch.cuda.current_stream(dev).cuda_stream
o = torch.from_numpy(testfactory.random_square(k, 0)).to(dev)
e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
r = torch.empty(W * 90, dtype=torch.uint8, device=dev)
c = torch.empty(W * 90, dtype=torch.uint8, device=dev)
g = torch.empty(32, dtype=torch.uint8, device=dev)
e.view(W, W, 512)[:k, :k] = o.view(k, k, 512)


def packed():
    ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(), None, s)


def inplace():
    ctx.extend_dah_inplace_device(k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(), None, s)


for rnd in range(4):
    for name, f in (("inplace", inplace), ("packed", packed)):
        f()
        torch.cuda.synchronize(dev)
        a = time.perf_counter()
        for _ in range(10):
            f()
        torch.cuda.synchronize(dev)
        print(rnd, name, round(1e3 * (time.perf_counter() - a) / 10, 4), "ms", flush=True)
