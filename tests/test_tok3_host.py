"""The host tokeniser (tok3.cpp tok3_tokenise: trie search, token streams)
on the CPU, no GPU call: digests of its token streams on synthetic and
fixture name blocks against tests/golden/tok3_digests.json, written by the
build the GPU tests pinned byte for byte against the reference
(tests/test_tok3_gpu.py); a tokeniser change that alters any stream fails
here before it reaches a GPU."""
import ctypes as C
import json
import os
import sys

import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_tok3_digests as M  # noqa: E402

SO = os.path.join(os.path.dirname(HERE), "fqzcomp5_amd", "libfqz5_mi355x.so")


@pytest.mark.skipif(not os.path.exists(SO), reason="library not built")
def test_token_stream_digests():
    so = C.CDLL(SO)
    want = json.load(open(os.path.join(HERE, "golden", "tok3_digests.json")))
    got_cases = M.cases()
    assert set(got_cases) == set(want)
    for k, data in got_cases.items():
        for lv, d in want[k].items():
            assert f"{M.digest(so, data, int(lv)):016x}" == d, (k, lv)
