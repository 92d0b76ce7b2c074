import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    # the oracle's countWithinDistance may use several host threads (integer sums: same counts);
    # at most 16 (the GPU box's CPU share)
    try:
        from oracle import oracle as O
        O.set_threads(min(16, os.cpu_count() or 1))
    except Exception:  # (oracle not built yet: its tests build it)
        pass
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device; runs the HIP path")
    config.addinivalue_line("markers", "slow: long-running (large clouds)")


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN


@pytest.fixture(scope="session")
def gpu_ctx():
    """One HIP context for the whole GPU session (no CPU fallback: fails if no device)."""
    from dialog_amd import Context
    ctx = Context(0)
    yield ctx
    ctx.close()
