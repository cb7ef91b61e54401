import json
import os
import sys

import numpy as np
import pytest

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs the HIP kernels")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def corpus():
    with np.load(os.path.join(GOLDEN, "corpus.npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def kat():
    return load_json("kat.json")["vectors"]


@pytest.fixture(scope="session")
def errors():
    return load_json("errors.json")


@pytest.fixture(scope="session")
def digests():
    return load_json("digests.json")["configs"]


@pytest.fixture(scope="session")
def codec():
    """One HIP context for the whole GPU session (tests run in one process)."""
    import torch
    from nghttp3_amd import HuffmanBatchCodec
    assert torch.cuda.is_available(), "gpu tests need a HIP device"
    c = HuffmanBatchCodec(device=0)
    yield c
    c.close()


def strings_of(plain, off, ln):
    return [plain[int(o):int(o) + int(n)].tobytes() for o, n in zip(off, ln)]
