import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
# a fault in the library's host code prints its native call stack
# (capi.cpp's env-gated SIGSEGV handler, read when the library loads)
os.environ.setdefault("FQZ5_SEGV_TRACE", "1")


def pytest_configure(config):
    config.addinivalue_line(
        "markers", "gpu: needs an MI355X (run on the GPU box via gpurun)")
    # torch's wheel bundles its own HIP runtime next to the one the library
    # links (/opt/rocm): whichever initialises the device second still works
    # only if torch went first, so sessions start torch's runtime before
    # any test loads the library (a no-op without a GPU)
    import torch
    if torch.cuda.is_available():
        torch.cuda.init()


@pytest.fixture(scope="session")
def golden_rans():
    """The reference-generated rANS vectors (tests/golden/make_golden.py)."""
    import json
    g = os.path.join(ROOT, "tests", "golden")
    man = json.load(open(os.path.join(g, "rans.json")))
    blob_in = open(os.path.join(g, "rans_inputs.bin"), "rb").read()
    blob_out = open(os.path.join(g, "rans_outputs.bin"), "rb").read()
    inputs = {k: blob_in[o:o + n] for k, (o, n, _) in man["inputs"].items()}
    cases = []
    for c in man["cases"]:
        exp = None
        if "off" in c:
            exp = blob_out[c["off"]:c["off"] + c["len"]]
        cases.append((c["input"], c["order"], c["len"], c["md5"], exp))
    return inputs, cases
