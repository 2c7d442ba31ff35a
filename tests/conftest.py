import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


def pytest_collection_modifyitems(session, config, items):
    """Device-pointer tests hand torch tensors to the C-ABI.  torch must bring up its HIP
    runtime before libptv_amd.so does (as bench.py does): a process whose first HIP call
    came from the library sees no GPU through torch afterwards."""
    if any(it.get_closest_marker("gpu") for it in items):
        try:
            import torch

            if torch.cuda.is_available():
                torch.cuda.init()
        except Exception:
            pass


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
