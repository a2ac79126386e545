"""The tok3 trie search on the GPU (tok3_search.hip, tok3_search_batch):
for every name of a batch of name blocks, search_trie's result
(tokenise_name3.c:591-695) equals the host trie's (tok3.cpp Trie::search,
whose token streams tests/test_tok3_host.py pins) -- fqz5_tok3_search_check
runs both and counts the names that differ.  Blocks: the tokeniser digest
cases, and constructed ones for each branch of the search: names that are
prefixes of earlier names, duplicates, empty names, '\\n' terminators, the
PacBio / IonTorrent / ONT uuid / Illumina formats of name_format, and the
same block twice in one batch (blocks must not see each other's names)."""
import ctypes as C
import os
import random
import sys

import pytest

from fqzcomp5_amd import lib

pytestmark = pytest.mark.gpu
HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "golden"))
import make_tok3_digests as M  # noqa: E402


@pytest.fixture(scope="module")
def so():
    if not lib.device_ok():
        pytest.fail("no GPU: " + lib.last_error())
    s = lib.load()
    s.fqz5_tok3_search_check.restype = C.c_longlong
    s.fqz5_tok3_search_check.argtypes = [C.c_char_p, C.POINTER(C.c_uint32), C.c_int, C.c_int]
    return s


def check(so, blocks, split=0):
    data = b"".join(blocks)
    lens = (C.c_uint32 * len(blocks))(*[len(b) for b in blocks])
    return so.fqz5_tok3_search_check(data, lens, len(blocks), split)


def constructed(seed):
    rng = random.Random(seed)
    names = []
    alpha = "AB:_-./ 0123456789"
    for i in range(4000):
        r = rng.random()
        if names and r < 0.15:
            names.append(rng.choice(names))                          # duplicate
        elif names and r < 0.3:
            p = rng.choice(names)
            names.append(p[:rng.randrange(0, len(p) + 1)])           # a prefix of an earlier one
        elif names and r < 0.45:
            p = rng.choice(names)
            names.append(p + "".join(rng.choice(alpha) for _ in range(rng.randrange(1, 6))))
        elif r < 0.5:
            names.append("")
        elif r < 0.6:
            names.append("m%06d_%06d_%s/%d/%d_%d" % (rng.randrange(10**6), rng.randrange(10**6),
                                                     "x" * 46, rng.randrange(99), rng.randrange(9),
                                                     rng.randrange(9)))   # PacBio, > 70 bytes
        elif r < 0.7:
            names.append("%05d:%05d:%05d" % (rng.randrange(10**5), rng.randrange(10**5),
                                             rng.randrange(10**5)))       # IonTorrent, 17 bytes
        elif r < 0.8:
            h = "%032x" % rng.getrandbits(128)
            names.append("%s-%s-%s-%s-%s%s" % (h[:8], h[8:12], h[12:16], h[16:20], h[20:],
                                               rng.choice(["", " runid=1", "_x"])))   # ONT uuid
        else:
            names.append("A00%d:%d:H%s:%d:%d:%d:%d%s" % (
                rng.randrange(9), rng.randrange(99), "X" * rng.randrange(1, 4), rng.randrange(1, 5),
                rng.randrange(1101, 1120), rng.randrange(1000, 1010), rng.randrange(100000),
                rng.choice(["", " 1:N:0:ACGT", "/1"])))                   # Illumina
    sep = [rng.choice([b"\0", b"\n"]) for _ in names]
    return b"".join(n.encode() + s for n, s in zip(names, sep))


def test_digest_cases(so):
    cases = M.cases()
    for k, data in cases.items():
        assert check(so, [data]) == 0, k


def test_constructed_blocks(so):
    for seed in range(3):
        assert check(so, [constructed(seed)]) == 0, seed


def test_batch_of_blocks_independent(so):
    a, b = constructed(7), constructed(8)
    assert check(so, [a, b, a, b[: len(b) // 2] + b"\0", a]) == 0


def test_refused_block(so):
    # a tab ends a name and is no terminator: the tokenise loop fails, the
    # batch leaves that block to the host (-1 - index)
    assert check(so, [b"ab\0cd\0", b"a\tb\0"]) == -2


def test_split_mode(so):
    """TOK3_n_LZP sections: the read ids searched in place in the name
    section (a space or tab ends the id, a "/1" or "/2" goes, a leading space
    of the section's first name does not count) against the host trie over
    name_split's ids."""
    cases = M.cases()
    secs = [v for k, v in cases.items() if not k.endswith("_ids") and v.endswith(b"\0")]
    assert check(so, secs, split=1) == 0
    rng = random.Random(5)
    names = []
    for i in range(3000):
        base = rng.choice(["r%d" % rng.randrange(500), "A1:2:%d" % rng.randrange(50), "", "x/1",
                           "/2", "q/3", "p/1/2"])
        tail = rng.choice(["", " c1", "\tc2", "/1", "/2", "/1 x", "/2\ty", " ", "\t"])
        names.append(base + tail)
    blk = b"".join(n.encode() + b"\0" for n in names)
    assert check(so, [blk, b" lead\0b c\0", blk], split=1) == 0
    # a tab at the section's first byte stays in the first id, which the
    # tokenise loop then refuses (the host split + trie refuse it too)
    assert check(so, [b"\tx\0y\0"], split=1) == -1
    # a '\n' in a section: the host split keeps it in the id (refused here)
    assert check(so, [b"a\nb\0c\0"], split=1) == -1
