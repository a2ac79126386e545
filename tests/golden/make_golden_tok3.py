"""Generate the tok3 name-tokeniser golden vectors from the compiled
reference (oracle/_ref/libhtsref.so: tokenise_name3.c's own
tok3_encode_names over the reference rANS 4x16 / arith_dynamic, built by
oracle/Makefile from /root/reference).

Inputs are regenerated from tests/tok3_cases.py (seeded).  Per case and
level (rANS levels 1-9, arith at levels 1 and 3) this stores the stream
length and md5 and last_start; streams of at most 20000 bytes are kept in
tok3_small.bin for decode tests.  Run from the repo root:
python tests/golden/make_golden_tok3.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from tok3_cases import cases, bad_cases  # noqa: E402
from oracle import binding  # noqa: E402

SETTINGS = [(lv, 0) for lv in (1, 3, 5, 7, 9)] + [(1, 1), (3, 1)]


def main():
    ref = binding.ref()
    out, blob = [], bytearray()
    for name, data in cases():
        for lv, ar in SETTINGS:
            r = ref.tok3_encode(data, lv, ar)
            assert r is not None, (name, lv, ar)
            z, ls = r
            dec = ref.tok3_decode(z)
            exp = data[:ls].replace(b"\n", b"\0")
            assert dec == exp, (name, lv, ar)
            rec = {"case": name, "level": lv, "arith": ar, "len": len(z),
                   "md5": hashlib.md5(z).hexdigest(), "last_start": ls, "off": None}
            if len(z) <= 20000:
                rec["off"] = len(blob)
                blob += z
            out.append(rec)
    for name, data in bad_cases():
        assert ref.tok3_encode(data, 5, 0) is None, name
    json.dump(out, open(os.path.join(HERE, "tok3.json"), "w"), indent=0)
    open(os.path.join(HERE, "tok3_small.bin"), "wb").write(bytes(blob))
    print(len(out), "vectors,", len(blob), "bytes of small outputs")


if __name__ == "__main__":
    main()
