"""fqz5file.compress_file / decompress_file on a 1 GB synthetic FASTQ file
(the bench's dropin_cli.gpu_file_path item alone): round trip and times."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from fqzcomp5_amd import fqz5file, synth  # noqa: E402

gb = float(sys.argv[1]) if len(sys.argv) > 1 else 1.0
level = int(sys.argv[2]) if len(sys.argv) > 2 else 3
r = synth.illumina(int(gb * 1e9 / 358), seed=1)
with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
    src, out, back = (os.path.join(td, n) for n in ("in.fastq", "out.fqz5", "back.fastq"))
    n = synth.write_fastq(r, src)
    reps = int(sys.argv[3]) if len(sys.argv) > 3 else 2
    for rep in range(reps):
        for pth in (out, back):          # fresh outputs, as the bench's
            if os.path.exists(pth):
                os.unlink(pth)
        t0 = time.perf_counter()
        fqz5file.compress_file(src, out, level)
        t1 = time.perf_counter()
        fqz5file.decompress_file(out, back)
        t2 = time.perf_counter()
        same = open(back, "rb").read() == open(src, "rb").read()
        print(f"file path -{level} {n/1e9:.2f} GB: enc {t1-t0:.3f} s ({n/(t1-t0)/1e6:.0f} MB/s), "
              f"dec {t2-t1:.3f} s ({n/(t2-t1)/1e6:.0f} MB/s), roundtrip {same}", flush=True)
        assert same
