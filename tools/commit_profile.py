#!/usr/bin/env python3
"""Run only the blob-commitment bench extra (for rocprofv3 kernel traces)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import json  # noqa: E402

import torch  # noqa: E402

import bench  # noqa: E402
from celestia_da import Context  # noqa: E402

dev = torch.device("cuda", 0)
ctx = Context(0)
stream = torch.cuda.current_stream(dev).cuda_stream
print(json.dumps(bench.blob_commitments(ctx, dev, stream, reps=int(os.environ.get("REPS", "10")))))
