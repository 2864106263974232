import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "celestia-app_amd")
ORACLE = os.path.join(ROOT, "oracle")
for p in (PKG, ORACLE, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP path)")


@pytest.fixture(scope="session")
def ctx():
    import celestia_da
    return celestia_da.default_context()


def pytest_runtest_makereport(item, call):
    """Keep the full text of every failing GPU test (the engine's error message
    names the stages enqueued since the context's work was last seen
    complete), so a fault seen once is on record: gpurun_out/gpu_failures.log
    (merged back from the GPU box; copied into profiles/ when it happens)."""
    if call.excinfo is None or item.get_closest_marker("gpu") is None:
        return
    try:
        import datetime
        d = os.path.join(ROOT, "gpurun_out")
        os.makedirs(d, exist_ok=True)
        with open(os.path.join(d, "gpu_failures.log"), "a") as f:
            f.write(f"==== {datetime.datetime.now().isoformat()} {item.nodeid} ({call.when})\n")
            f.write(f"{call.excinfo.typename}: {call.excinfo.value}\n")
            for e in call.excinfo.traceback:   # this repository's frames only
                path = str(e.path)
                if path.startswith(ROOT) and "/site-packages/" not in path:
                    f.write(f"  {os.path.relpath(path, ROOT)}:{e.lineno + 1}: {str(e.statement).strip()}\n")
    except Exception:
        pass
