"""Exercise bench.config5 on ONE GPU (world 1, gloo process group): the split
kernels, the orchestration and rank-0's check against the single-GPU path.
(N>1 runs with RCCL only in the driver's multi-GPU bench.)"""
import json
import os
import sys

import torch
import torch.distributed as dist

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
from celestia_da import Context  # noqa: E402

os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
os.environ.setdefault("MASTER_PORT", "29531")
dist.init_process_group("gloo", rank=0, world_size=1)
dev = torch.device("cuda", 0)
torch.cuda.set_device(dev)
print(json.dumps(bench.config5(Context(0), dev, 0, 1, 512)))
dist.destroy_process_group()
