import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import gome_amd  # noqa: E402,F401  (before torch: the HIP runtime's hardware-queue count)

# One HIP runtime per process: torch bundles its own libamdhip64.so.7 (same SONAME as
# /opt/rocm's); importing torch first makes libgome.so bind to that one too, so tests
# that hand torch device buffers to the engine share one runtime.
try:
    import torch  # noqa: F401
except Exception:  # pragma: no cover
    torch = None



def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    # GOME_TEST_POISON=1: every engine a test creates starts its device buffers 0xA5-filled
    # (GOME_FLAG_POISON), so a kernel reading scratch it never wrote shows up in the whole suite
    if os.environ.get("GOME_TEST_POISON") == "1":
        from gome_amd import abi
        init = abi.Engine.__init__

        def poisoned(self, *a, flags: int = 0, **kw):
            init(self, *a, flags=flags | abi.GOME_FLAG_POISON, **kw)

        abi.Engine.__init__ = poisoned


@pytest.fixture(scope="session", autouse=True)
def _built():
    from gome_amd.build import build_all
    build_all()
