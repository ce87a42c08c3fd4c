import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tests"))

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device")


def load_fixture(name):
    """(Rows, vids, schema_dict, npz) of a committed golden fixture."""
    import edgestore as es
    npz = np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False)
    with open(os.path.join(GOLDEN, name + ".schema.json")) as f:
        sd = json.load(f)
    return es.Rows.load(npz), npz["vids"], sd, npz


@pytest.fixture(scope="session")
def gpu_available():
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:
        return False
