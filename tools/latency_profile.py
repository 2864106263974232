"""Single-square extend+DAH latency (config 2): wall per call vs GPU kernel time (run under rocprofv3)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "celestia-app_amd"))
from celestia_da import Context, testfactory  # noqa: E402

k = int(sys.argv[1]) if len(sys.argv) > 1 else 128
W = 2 * k
ctx = Context(0)
dev = torch.device("cuda", 0)
o = torch.from_numpy(testfactory.random_square(k, 0)).to(dev)
e = torch.empty(W * W * 512, dtype=torch.uint8, device=dev)
r = torch.empty(W * 90, dtype=torch.uint8, device=dev)
c = torch.empty(W * 90, dtype=torch.uint8, device=dev)
g = torch.empty(32, dtype=torch.uint8, device=dev)
st = torch.empty(1, dtype=torch.int32, device=dev)
s = torch.cuda.current_stream(dev).cuda_stream
lat = []
for i in range(30):
    torch.cuda.synchronize(dev)
    a = time.perf_counter()
    ctx.extend_dah_device(o.data_ptr(), k, 1, e.data_ptr(), r.data_ptr(), c.data_ptr(), g.data_ptr(), st.data_ptr(), s)
    b = time.perf_counter()
    torch.cuda.synchronize(dev)
    lat.append((b - a, time.perf_counter() - a))
lat = lat[5:]
print("enqueue_ms", 1e3 * float(np.median([x[0] for x in lat])), "wall_ms", 1e3 * float(np.median([x[1] for x in lat])))
