"""Seeded LZP inputs (lzp16e.c; fqzcomp5.c's LZP3 sequence method) shared by
the golden-vector generator and the tests: empty and tiny inputs, random
ACGT (few short matches), repeated reads (long matches, 2-byte lengths),
runs longer than the 65535 match cap, raw and escaped marker bytes (233 /
234) with and without a prediction, and random bytes."""
import random


def cases():
    rng = random.Random(2024)
    out = [("empty", b""), ("one", b"A"), ("two", b"AC"), ("three", b"ACG"),
           ("four", b"ACGT"), ("five", b"ACGTA"), ("run7", b"A" * 7)]
    out.append(("acgt_20k", bytes(rng.choice(b"ACGT") for _ in range(20000))))
    out.append(("acgtn_60k", bytes(rng.choice(b"ACGTN") if rng.random() < .99 else 78
                                   for _ in range(60000))))
    read = bytes(rng.choice(b"ACGT") for _ in range(150))
    out.append(("amplicon", read * 200))
    reads = [bytes(rng.choice(b"ACGT") for _ in range(150)) for _ in range(20)]
    out.append(("pool", b"".join(rng.choice(reads) for _ in range(400))))
    out.append(("run_200k", b"A" * 200000))
    out.append(("period3_100k", b"ACG" * 33334))
    out.append(("markers", bytes([233, 234] * 600)))
    out.append(("marker_mix", bytes(rng.choice([233, 234, 65, 67]) for _ in range(40000))))
    out.append(("bytes_30k", bytes(rng.randrange(256) for _ in range(30000))))
    # long repeats with mutations: match lengths around 255/256 and 65535
    base = bytes(rng.choice(b"ACGT") for _ in range(70000))
    mut = bytearray(base)
    for p in (255 + 4, 256 + 700, 66000):
        mut[p] = ord("N")
    out.append(("mutated_copy", base + bytes(mut)))
    return out
