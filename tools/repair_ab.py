#!/usr/bin/env python3
"""Only the eds_repair bench extra (A/B of libcda builds via CDA_LIB)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))
import bench  # noqa: E402
from celestia_da import Context  # noqa: E402

ctx = Context(0)
print(os.environ.get("CDA_LIB", "default"), json.dumps(bench.eds_repair(ctx, reps=int(os.environ.get("REPS", "9")))))
