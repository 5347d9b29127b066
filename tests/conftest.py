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
    """Build (incrementally) unless the library already carries the checked-out sources' hash; then
    refuse to test a library built from other sources (lh2_version() "srchash=...")."""
    from lighthouse2_amd import build_info
    orc = ROOT / "oracle" / "liboracle.so"
    want = build_info.source_hash()
    if build_info.library_hash() != want or not orc.exists():
        import __graft_entry__
        __graft_entry__.build()
    got = build_info.library_hash()
    if got != want:
        raise RuntimeError(f"libRenderCore_MI355X.so srchash={got} but the sources hash to {want}")
    print(f"lighthouse2_amd: libRenderCore_MI355X.so srchash={got} (matches sources)", file=sys.stderr)


_ensure_built()


def pytest_report_header(config):
    from lighthouse2_amd import build_info
    return f"libRenderCore_MI355X.so srchash={build_info.library_hash()} sources={build_info.source_hash()}"


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
