"""Run only bench.py's host-buffer extra (cgo drop-in path: host ODS in,
host EDS / roots out).  CDA_HOST_THREADS picks the host-side Q0 copy's
thread count (read when the library loads)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "celestia-app_amd"))

import bench  # noqa: E402
from celestia_da import Context  # noqa: E402

ctx = Context(0)
r = bench.host_buffer_rates(ctx, 128)
print(json.dumps({k: v for k, v in r.items() if k != "note"}))
