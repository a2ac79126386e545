"""Regression digests of the host tokeniser's token streams
(fqz5_tok3_tokenise_digest) on synthetic and fixture name blocks, written
by the build whose tok3 output the GPU tests pinned byte for byte against
the reference (tests/test_tok3_gpu.py, tests/test_trial_parity_gpu.py).
Usage: python tests/golden/make_tok3_digests.py  (writes tok3_digests.json)"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))


def cases():
    from fqzcomp5_amd import synth
    out = {}
    gens = {"illumina": lambda: synth.illumina(20000, seed=1, with_names=True),
            "novaseq": lambda: synth.novaseq(20000, seed=2, with_names=True),
            "ont": lambda: synth.ont(300, seed=3, with_names=True),
            "hifi": lambda: synth.hifi(100, seed=4, with_names=True)}
    for k, g in gens.items():
        buf, _ = synth.all_names(g())
        full = bytes(buf)
        out[k] = full
        out[k + "_ids"] = b"\0".join(n.split(b" ")[0] for n in full.split(b"\0")[:-1]) + b"\0"
    for f in sorted(os.listdir(os.path.join(HERE, "fastq"))):
        lines = open(os.path.join(HERE, "fastq", f), "rb").read().split(b"\n")
        names = [ln[1:].rstrip(b"\r") for ln in lines[0::4] if ln.startswith(b"@")]
        if names:
            out["fastq/" + f] = b"\0".join(names) + b"\0"
    return out


def digest(so, data: bytes, level: int) -> int:
    import ctypes as C
    so.fqz5_tok3_tokenise_digest.restype = C.c_ulonglong
    so.fqz5_tok3_tokenise_digest.argtypes = [C.c_char_p, C.c_int, C.c_int]
    return int(so.fqz5_tok3_tokenise_digest(data, len(data), level))


if __name__ == "__main__":
    import ctypes as C
    so = C.CDLL(os.path.join(os.path.dirname(os.path.dirname(HERE)), "fqzcomp5_amd",
                             "libfqz5_mi355x.so"))
    res = {k: {str(lv): f"{digest(so, v, lv):016x}" for lv in (3, 9)} for k, v in cases().items()}
    json.dump(res, open(os.path.join(HERE, "tok3_digests.json"), "w"), indent=1, sort_keys=True)
    print(len(res), "cases")
