"""Generate the sequence context model golden vectors from the compiled
reference (oracle/_ref/libfqz5ref.so: fqzcomp5.c's own encode_seq /
decode_seq, built by oracle/Makefile from /root/reference).

Inputs are regenerated from tests/seq_cases.py (seeded); this script stores
for every (case, method) the output length and md5, and the bytes of the
small outputs (seq_small.bin) for decode tests.
Run from the repo root: python tests/golden/make_golden_seq.py
"""
import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

from seq_cases import METHODS, cases  # noqa: E402
from oracle import binding  # noqa: E402


def main():
    ref = binding.seq_ref()
    out, blob = [], bytearray()
    for name, seq, lens in cases():
        for meth, k, both in METHODS:
            c = ref.encode(seq, lens, both, k)
            rec = {"case": name, "method": meth, "k": k, "both": both, "len": len(c),
                   "md5": hashlib.md5(c).hexdigest(), "off": None}
            if len(c) <= 40000:
                rec["off"] = len(blob)
                blob += c
            assert ref.decode(c, lens, both, k, len(seq)) == seq, (name, meth)
            out.append(rec)
    json.dump(out, open(os.path.join(HERE, "seq.json"), "w"), indent=0)
    open(os.path.join(HERE, "seq_small.bin"), "wb").write(bytes(blob))
    print(len(out), "vectors,", len(blob), "bytes of small outputs")


if __name__ == "__main__":
    main()
