"""Generate the fqzcomp_qual golden vectors from the compiled reference
(oracle/_ref/libhtsref.so, built by oracle/Makefile from /root/reference).

Inputs are regenerated from tests/fqz_cases.py (seeded); this script stores
for every (case, strat) the expected output length and md5, and the full
output bytes of the small ones (fqz_small.bin) for decode tests.
Run from the repo root: python tests/golden/make_golden_fqz.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from fqz_cases import STRATS, cases  # noqa: E402
from oracle import binding  # noqa: E402


def main():
    ref = binding.ref()
    out, blob = [], bytearray()
    for name, q, lens, flags, seq in cases():
        for st in STRATS:
            c = ref.fqz_compress(q, lens.copy(), flags.copy(), st, seq)
            rec = {"case": name, "strat": st, "len": len(c),
                   "md5": hashlib.md5(c).hexdigest(), "off": None}
            if len(c) <= 40000:
                rec["off"] = len(blob)
                blob += c
            back = ref.fqz_decompress(c, lens.copy(), flags.copy(), seq)
            assert back == q, (name, st)
            out.append(rec)
    json.dump(out, open(os.path.join(HERE, "fqz.json"), "w"), indent=0)
    open(os.path.join(HERE, "fqz_small.bin"), "wb").write(bytes(blob))
    print(len(out), "vectors,", len(blob), "bytes of small outputs")


if __name__ == "__main__":
    main()
