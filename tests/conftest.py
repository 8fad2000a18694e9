import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
if str(ROOT) not in sys.path:
    sys.path.insert(0, str(ROOT))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built libirx.so")
    config.addinivalue_line("markers", "slow: long-running CPU test")


@pytest.fixture(scope="session")
def device():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda:0")


REFERENCE = Path("/root/reference")


@pytest.fixture(autouse=True)
def _restore_options():
    """Every test leaves the engine's runtime options (irx_set_option) as it found them: a snapshot before the test,
    restored after it (a toggle restored to a non-default value changed what later tests ran)."""
    from image_restoration_and_enhancement_amd import _lib as L
    try:
        L.load()          # (loaded before the snapshot: the first test to load the library is restored too)
    except L.IrxError:
        pass
    before = L.options() if L._lib is not None else None
    yield
    if before is None or L._lib is None:
        return
    for k, v in L.options().items():
        if before.get(k, v) != v:
            L.call("irx_set_option", k.encode(), before[k])
