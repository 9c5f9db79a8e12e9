import os
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "sac-agent_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device)")


def golden(name: str) -> dict:
    """A fixture's arrays, decompressed once (an NpzFile re-reads its member per access)."""
    with np.load(os.path.join(GOLDEN, name), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


def seeded_fixtures():
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("seeded_"))


def long_fixtures():
    """The 10 000-step scripted runs (make_golden.py run_long)."""
    return sorted(f for f in os.listdir(GOLDEN) if f.startswith("long_"))


@pytest.fixture(scope="session")
def built_lib():
    import __graft_entry__
    __graft_entry__.build()
    from sacenv import _lib
    return _lib.load()


@pytest.fixture(scope="session")
def gpu():
    import torch
    if not torch.cuda.is_available():
        pytest.fail("GPU test selected but no HIP device is visible")
    return torch.device("cuda:0")
