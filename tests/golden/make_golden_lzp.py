"""Generate the LZP / LZP3 golden vectors from the compiled reference
(oracle/_ref/libhtsref.so: lzp16e.c's own lzp / unlzp and the reference
rANS order 5 for LZP3, built by oracle/Makefile from /root/reference).

Inputs are regenerated from tests/lzp_cases.py (seeded); this script stores
per case the lzp output length and md5, the LZP3 stream length and md5, and
the bytes of the small outputs (lzp_small.bin) for decode tests.
Run from the repo root: python tests/golden/make_golden_lzp.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from lzp_cases import cases  # noqa: E402
from oracle import binding  # noqa: E402


def main():
    ref = binding.ref()
    out, blob = [], bytearray()
    for name, data in cases():
        z = ref.lzp(data)
        c = ref.lzp3_compress(data)
        assert ref.unlzp(z, len(data) + 64) == data, name
        rec = {"case": name, "n": len(data), "lzp_len": len(z),
               "lzp_md5": hashlib.md5(z).hexdigest(), "lzp3_len": len(c),
               "lzp3_md5": hashlib.md5(c).hexdigest(), "off": None}
        if len(c) <= 20000:
            rec["off"] = len(blob)
            blob += c
        out.append(rec)
    json.dump(out, open(os.path.join(HERE, "lzp.json"), "w"), indent=0)
    open(os.path.join(HERE, "lzp_small.bin"), "wb").write(bytes(blob))
    print(len(out), "vectors,", len(blob), "bytes of small outputs")


if __name__ == "__main__":
    main()
