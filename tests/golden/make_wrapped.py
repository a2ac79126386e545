"""Reference md5s for wrapped (multi-line) FASTQ (tests/wrapped_cases.py):
the reference CLI as compiled from /root/reference (oracle/_ref/fqzcomp5,
-t1, 1 MB blocks) codes each case at -1 / -3 / -5; stored per case and level:
the .fqz5 md5 and length, and the md5 and length of its `-d` output (kseq's
records written 4-line, fqzcomp5.c:3441-3480).
Run from the repo root: python tests/golden/make_wrapped.py
"""
import hashlib
import json
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.dirname(HERE))
sys.path.insert(0, ROOT)

from wrapped_cases import CASES  # noqa: E402

CLI = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")


def main():
    out = []
    with tempfile.TemporaryDirectory() as td:
        for name, gen in CASES.items():
            text = gen()
            src = os.path.join(td, name + ".fastq")
            open(src, "wb").write(text)
            for level in (1, 3, 5):
                z, back = os.path.join(td, "o.fqz5"), os.path.join(td, "o.fastq")
                subprocess.run([CLI, f"-{level}", "-t1", "-b", "1M", src, z], check=True,
                               capture_output=True)
                subprocess.run([CLI, "-d", "-t1", z, back], check=True, capture_output=True)
                zb, bb = open(z, "rb").read(), open(back, "rb").read()
                out.append({"case": name, "level": level, "fastq_md5": hashlib.md5(text).hexdigest(),
                            "fqz5_len": len(zb), "fqz5_md5": hashlib.md5(zb).hexdigest(),
                            "dec_len": len(bb), "dec_md5": hashlib.md5(bb).hexdigest()})
                print(name, level, len(text), "->", len(zb), "->", len(bb))
    json.dump(out, open(os.path.join(HERE, "wrapped.json"), "w"), indent=0)


if __name__ == "__main__":
    main()
