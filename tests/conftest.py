import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdeltagpu on cuda:0)")


@pytest.fixture(scope="session")
def engine():
    import torch
    from delta_crdt_ex_amd.store import Engine
    if not torch.cuda.is_available():
        pytest.fail("gpu tests need an MI355X: torch.cuda.is_available() is False")
    e = Engine(0)
    yield e
    e.close()
