import os
import pathlib
import sys

import pytest

try:  # torch first: the render core then binds to the same HIP runtime (one libamdhip64.so.7)
    import torch  # noqa: F401
except ImportError:  # pragma: no cover
    torch = None

ROOT = pathlib.Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long-running test")


def _ensure_built():
    lib = ROOT / "lighthouse2_amd" / "libRenderCore_MI355X.so"
    orc = ROOT / "oracle" / "liboracle.so"
    if not lib.exists() or not orc.exists():
        import __graft_entry__
        __graft_entry__.build()


_ensure_built()


@pytest.fixture(scope="session")
def core():
    """One MI355X render core for the whole GPU test session (single process on the card)."""
    from lighthouse2_amd.core import RenderCore
    c = RenderCore(device=int(os.environ.get("LH2_TEST_DEVICE", "0")))
    yield c
    c.close()


@pytest.fixture()
def fresh_core():
    from lighthouse2_amd.core import RenderCore
    c = RenderCore(device=int(os.environ.get("LH2_TEST_DEVICE", "0")))
    yield c
    c.close()
