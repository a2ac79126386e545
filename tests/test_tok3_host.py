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


@pytest.mark.skipif(not os.path.exists(SO), reason="library not built")
def test_pipelined_search_same_streams():
    """tok3_tokenise(pipelined): the trie searches on a second thread ahead
    of the coding (names.cpp uses it when sections are fewer than host
    threads) give the same token streams."""
    so = C.CDLL(SO)
    f = so.fqz5_tok3_tokenise_digest_mode
    f.restype = C.c_ulonglong
    f.argtypes = [C.c_char_p, C.c_int, C.c_int, C.c_int]
    want = json.load(open(os.path.join(HERE, "golden", "tok3_digests.json")))
    for k, data in M.cases().items():
        for lv, d in want[k].items():
            assert f"{f(data, len(data), int(lv), 1):016x}" == d, (k, lv)
    bad = b"a\0b\tc\0"                         # a tab ends a name: NULL both ways
    assert f(bad, len(bad), 3, 1) == f(bad, len(bad), 3, 0) == 0
