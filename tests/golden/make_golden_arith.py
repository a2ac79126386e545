#!/usr/bin/env python3
"""arith_compress_to golden vectors from the compiled reference
(oracle/_ref/libhtsref.so).  Run here:

    make -C oracle && python tests/golden/make_golden_arith.py

Inputs are the committed rANS golden inputs (rans_inputs.bin, rans.json).
Written: arith.json (manifest) and arith_outputs.bin (outputs up to
SMALL_OUT bytes verbatim; larger ones by length + md5).  Capacity cases
record whether a caller buffer of a given size gives NULL (EXT is only
tried with out == NULL: the reference frees the output buffer on that
path)."""
from __future__ import annotations

import hashlib
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import binding  # noqa: E402

SMALL_OUT = 4000
ORDERS = [0, 1, 64, 65, 128, 129, 192, 193, 32, 16, 17, 4,
          8, 9, (2 << 8) | 8, (3 << 8) | 9, (7 << 8) | 8, (16 << 8) | 9,
          (4 << 8) | 0x48, (4 << 8) | 0x89, (150 << 8) | 9]


def main():
    man = json.load(open(os.path.join(HERE, "rans.json")))
    blob = open(os.path.join(HERE, "rans_inputs.bin"), "rb").read()
    ins = {k: blob[o:o + n] for k, (o, n, _) in man["inputs"].items()}
    ref = binding.ref()
    out = bytearray()
    cases, caps = [], []
    for name, data in ins.items():
        if len(data) > 300000:
            continue
        for od in ORDERS:
            r = ref.arith_compress(data, od)
            c = {"input": name, "order": od}
            if r is None:
                c["null"] = True
            else:
                c["len"] = len(r)
                c["md5"] = hashlib.md5(r).hexdigest()
                if len(r) <= SMALL_OUT:
                    c["off"] = len(out)
                    out += r
            cases.append(c)
    for name in ("pat_40", "pat_1000", "qual8_5000", "q40_20000"):
        data = ins[name]
        for od in (0, 1, 65, 129, 193, 9):
            full = ref.arith_compress(data, od)
            bound = ref.arith_compress_bound(len(data), od)
            for cap in sorted({1, len(full) - 1, len(full), len(full) + 1, bound - 1, bound}):
                if cap <= 0:
                    continue
                r = ref.arith_compress(data, od, cap=cap)
                caps.append({"input": name, "order": od, "cap": cap,
                             "null": r is None, "md5": None if r is None else
                             hashlib.md5(r).hexdigest()})
    json.dump({"cases": cases, "caps": caps}, open(os.path.join(HERE, "arith.json"), "w"),
              indent=0)
    open(os.path.join(HERE, "arith_outputs.bin"), "wb").write(bytes(out))
    print(len(cases), "cases,", len(caps), "capacity cases,", len(out), "bytes")


if __name__ == "__main__":
    main()
