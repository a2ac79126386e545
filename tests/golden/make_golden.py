#!/usr/bin/env python3
"""Generate byte-level golden vectors from the compiled reference.

Run HERE (where /root/reference and oracle/_ref exist):

    make -C oracle && python tests/golden/make_golden.py

The reference ships no byte-level vectors, so these
are produced by the reference itself (oracle/_ref/libhtsref.so, compiled
from /root/reference by oracle/Makefile).  Only data is committed: inputs,
expected outputs (or their md5 + length for large ones) and the manifest.

Files written next to this script:
  rans_inputs.bin   concatenated rANS test inputs
  rans_outputs.bin  concatenated expected outputs for the small cases
  rans.json         manifest {inputs: {name: [off, len, md5]},
                              cases: [{input, order, len, md5, off?}]}
  fqz_*.bin/json    fqz_compress vectors (see make_fqz()).
  fqz5/*.fqz5       whole-container files written by the reference binary.
"""
from __future__ import annotations

import hashlib
import json
import os
import subprocess
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from oracle import binding  # noqa: E402
from fqzcomp5_amd import synth  # noqa: E402

SMALL_OUT = 6000  # outputs up to this size are stored verbatim


def md5(b: bytes) -> str:
    return hashlib.md5(b).hexdigest()


def rans_inputs() -> dict[str, bytes]:
    ins: dict[str, bytes] = {}
    # SURVEY.md "worked stream anatomy": in[i] = i%7==0 ? 2 : i%3==0 ? 12 : 37
    pat = bytes(2 if i % 7 == 0 else 12 if i % 3 == 0 else 37
                for i in range(4096))
    for n in (0, 1, 2, 3, 4, 5, 7, 8, 9, 20, 21, 31, 32, 33, 40, 63, 64,
              100, 257, 1000, 1001, 1025, 4096):
        ins[f"pat_{n}"] = pat[:n]
    r = synth.illumina(2000, seed=11)
    q = r.qual.tobytes()
    for n in (999, 1000, 1001, 5000, 65537, 300000):
        ins[f"qual8_{n}"] = q[:n]
    r = synth.illumina(2000, seed=12, binned=False)
    q = r.qual.tobytes()
    for n in (1001, 20000, 100003, 300000):
        ins[f"q40_{n}"] = q[:n]
    s = r.seq.tobytes()
    for n in (997, 30000, 250001):
        ins[f"seq_{n}"] = s[:n]
    nv = synth.novaseq(400, seed=13).qual.tobytes()
    ins["nova_40000"] = nv[:40000]
    rng = np.random.default_rng(14)
    ins["rand_5000"] = rng.integers(0, 256, 5000, dtype=np.uint8).tobytes()
    ins["rand_70000"] = rng.integers(0, 256, 70000, dtype=np.uint8).tobytes()
    z = np.minimum(rng.zipf(1.3, 100000), 255).astype(np.uint8)
    ins["zipf_100000"] = z.tobytes()
    runs = np.repeat(rng.integers(0, 6, 6000).astype(np.uint8),
                     rng.integers(1, 20, 6000))
    ins["runs_%d" % len(runs)] = runs.tobytes()
    ins["const_100"] = b"\x07" * 100
    ins["const_5000"] = b"\x28" * 5000
    ins["two_3000"] = rng.choice(np.array([3, 9], np.uint8), 3000).tobytes()
    three = rng.choice(np.array([0, 1, 2], np.uint8), 2001,
                       p=[.8, .15, .05]).tobytes()
    ins["three_2001"] = three
    # 17 symbols: PACK rejected (>16)
    ins["sym17_3000"] = rng.integers(0, 17, 3000, dtype=np.uint8).tobytes()
    # 16 symbols: PACK 2/byte
    ins["sym16_3001"] = rng.integers(0, 16, 3001, dtype=np.uint8).tobytes()
    ins["sym5_777"] = rng.integers(40, 45, 777, dtype=np.uint8).tobytes()
    return ins


BASE_ORDERS = [0, 1, 4, 5, 64, 65, 68, 69, 128, 129, 132, 133,
               192, 193, 196, 197, 0x20, 0x21]
STRIPE_ORDERS = [(4 << 8) | 9, (8 << 8) | 9, (100 << 8) | 9,
                 (150 << 8) | 9, (250 << 8) | 9,
                 (4 << 8) | 8, (4 << 8) | 0x0d | 0x80,
                 (256 << 8) | 9,        # fixed_len 256 aliasing quirk
                 (300 << 8) | 9]        # fixed_len 300: N=44 + STRIPE_NO0


def make_rans():
    ref = binding.ref()
    ins = rans_inputs()
    blob_in = bytearray()
    manifest = {"inputs": {}, "cases": []}
    for name, data in ins.items():
        manifest["inputs"][name] = [len(blob_in), len(data), md5(data)]
        blob_in += data
    blob_out = bytearray()
    big = {"q40_300000", "qual8_300000", "seq_250001"}
    for name, data in ins.items():
        orders = list(BASE_ORDERS)
        if len(data) >= 20 and name not in ("zipf_100000",):
            orders += STRIPE_ORDERS
        if name in big:
            orders = [0, 1, 4, 5, 129, 193, (150 << 8) | 9]
        for order in orders:
            try:
                out = ref.rans_compress(data, order)
            except RuntimeError:
                continue
            back = ref.rans_uncompress(out)
            assert back == data, (name, order)
            case = {"input": name, "order": order, "len": len(out),
                    "md5": md5(out)}
            if len(out) <= SMALL_OUT:
                case["off"] = len(blob_out)
                blob_out += out
            manifest["cases"].append(case)
    with open(os.path.join(HERE, "rans_inputs.bin"), "wb") as f:
        f.write(blob_in)
    with open(os.path.join(HERE, "rans_outputs.bin"), "wb") as f:
        f.write(blob_out)
    with open(os.path.join(HERE, "rans.json"), "w") as f:
        json.dump(manifest, f, indent=0)
    print("rans: %d inputs (%d B), %d cases, %d B stored outputs"
          % (len(ins), len(blob_in), len(manifest["cases"]), len(blob_out)))


if __name__ == "__main__":
    what = sys.argv[1:] or ["rans"]
    if "rans" in what:
        make_rans()
