"""The streaming and multi-GPU file path on the GPU (fqzcomp5_amd/fqz5file.py;
VERDICT r02 items 4 and 5).

* windows: the input read in windows of whole records, the last block of a
  window carried into the next, the trial state carried across windows —
  the file equals the reference CLI's (-t1) byte for byte at -3/-5/-7 and
  for paired input, and decodes back in windows;
* ranks: two processes (gloo, both on this GPU) write the same file as one
  process, each coding its contiguous share of the blocks and its share of
  the trial's work candidates, and decode it back together;
* the -7 preset: a 1.1 GB ONT file in the preset's 500 MB blocks equals the
  reference CLI's -7 -t1 output (md5 recorded by tests/golden/make_golden_l7.py).
"""
import hashlib
import json
import os
import socket
import subprocess

import pytest
import torch.multiprocessing as mp

from fqzcomp5_amd import fqz5file, synth

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")
pytestmark = pytest.mark.gpu


def _cli(args, cwd=None):
    subprocess.run([CLI] + args, check=True, capture_output=True, cwd=cwd)


def _illumina(path, n=60000, seed=21):
    synth.write_fastq(synth.illumina(n, seed=seed, with_names=True), path)


@pytest.mark.parametrize("level", [3, 5, 7])
def test_windows_equal_cli(tmp_path, level):
    src = str(tmp_path / "in.fastq")
    _illumina(src)
    want, got, back = (str(tmp_path / x) for x in ("w.fqz5", "g.fqz5", "b.fastq"))
    _cli([f"-{level}", "-t1", "-b", "1M", src, want])
    # ~3 blocks per window: every window carries its last block over
    n = fqz5file.compress_file(src, got, level, blk_size=1_000_000, window_bytes=3_500_000)
    assert n == os.path.getsize(want)
    assert open(got, "rb").read() == open(want, "rb").read()
    assert fqz5file.decompress_file(got, back, window_bytes=1_500_000) == os.path.getsize(src)
    assert open(back, "rb").read() == open(src, "rb").read()


def test_windows_paired_equal_cli(tmp_path):
    r1, r2 = str(tmp_path / "r1.fastq"), str(tmp_path / "r2.fastq")
    a = synth.illumina(20000, seed=5, with_names=True)
    b = synth.illumina(20000, seed=6, with_names=True)
    synth.write_fastq(a, r1)
    synth.write_fastq(b, r2)
    want, got = str(tmp_path / "w.fqz5"), str(tmp_path / "g.fqz5")
    _cli(["-3", "-t1", "-b", "1M", r1, r2, want])
    fqz5file.compress_file(r1, got, 3, blk_size=1_000_000, src2=r2, window_bytes=2_000_000)
    assert open(got, "rb").read() == open(want, "rb").read()
    o1, o2 = str(tmp_path / "o1.fastq"), str(tmp_path / "o2.fastq")
    fqz5file.decompress_file(got, o1, dst2=o2, window_bytes=1_000_000)
    assert open(o1, "rb").read() == open(r1, "rb").read()
    assert open(o2, "rb").read() == open(r2, "rb").read()


def _rank(rank, world, port, args, q):
    import faulthandler
    import torch
    import torch.distributed as dist
    faulthandler.dump_traceback_later(120, exit=False)   # a hung rank shows where
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        src, dst, back, level, wb = args
        fqz5file.H2D[0] = 0
        n = fqz5file.compress_file(src, dst, level, blk_size=1_000_000, group=dist.group.WORLD,
                                   window_bytes=wb)
        h2d = fqz5file.H2D[0]
        m = fqz5file.decompress_file(dst, back, group=dist.group.WORLD, window_bytes=1_000_000)
        q.put((rank, n, m, h2d, None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, 0, 0, 0, repr(e)))
    finally:
        dist.destroy_process_group()


def _run_ranks(ps, q, wait=150):
    """Start the rank processes and collect one result from each; a rank
    that has not answered within `wait` seconds (under the GPU box's 180 s
    silence limit) fails the test, and every rank still alive at the end is
    killed, so no rank outlives its test (a lingering rank held the next
    test's rendezvous once)."""
    import queue
    for p in ps:
        p.start()
    out = []
    try:
        for _ in ps:
            try:
                out.append(q.get(timeout=wait))
            except queue.Empty:
                raise AssertionError(f"a rank did not answer within {wait} s; "
                                     f"the others answered {out}") from None
        return out
    finally:
        for p in ps:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("level", [5, 7])
def test_two_ranks_equal_one_process(tmp_path, level):
    """Two ranks write the one-process file byte for byte, each reading its
    share of every window once: a rank's host-to-device
    text is at most 0.6 x the file (its half, the trial blocks it shares,
    the ends of its last blocks), and the file decodes back on two ranks."""
    src = str(tmp_path / "in.fastq")
    _illumina(src, n=300000, seed=31)
    size = os.path.getsize(src)
    one, two, back = (str(tmp_path / x) for x in ("one.fqz5", "two.fqz5", "back.fastq"))
    fqz5file.compress_file(src, one, level, blk_size=1_000_000)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, 2, port, (src, two, back, level, 40_000_000), q))
          for r in range(2)]
    out = _run_ranks(ps, q)
    assert all(e is None for *_, e in out), out
    assert all(p.exitcode == 0 for p in ps)
    assert open(two, "rb").read() == open(one, "rb").read()
    assert open(back, "rb").read() == open(src, "rb").read()
    for rank, _, _, h2d, _ in out:
        assert h2d <= 0.6 * size, (rank, h2d, size)


def test_two_ranks_paired_small_windows(tmp_path):
    """Paired files on two ranks with windows of a few blocks (every window
    carries a block over, R1 and R2 cut at different bytes): the file equals
    the one-process file."""
    r1, r2 = str(tmp_path / "r1.fastq"), str(tmp_path / "r2.fastq")
    synth.write_fastq(synth.illumina(20000, seed=5, with_names=True), r1)
    synth.write_fastq(synth.novaseq(20000, seed=6, with_names=True), r2)
    one, two = str(tmp_path / "one.fqz5"), str(tmp_path / "two.fqz5")
    fqz5file.compress_file(r1, one, 3, blk_size=1_000_000, src2=r2)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_pairs, args=(r, 2, port, (r1, r2, two), q)) for r in range(2)]
    out = _run_ranks(ps, q)
    assert all(e is None for *_, e in out), out
    assert open(two, "rb").read() == open(one, "rb").read()


def _rank_pairs(rank, world, port, args, q):
    import faulthandler
    import torch
    import torch.distributed as dist
    faulthandler.dump_traceback_later(120, exit=False)   # a hung rank shows where
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.init()
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        r1, r2, dst = args
        fqz5file.compress_file(r1, dst, 3, blk_size=1_000_000, src2=r2, group=dist.group.WORLD,
                               window_bytes=3_000_000)
        q.put((rank, None))
    except Exception as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e)))
    finally:
        dist.destroy_process_group()


def _md5(path):
    h = hashlib.md5()
    with open(path, "rb") as f:
        for c in iter(lambda: f.read(1 << 24), b""):
            h.update(c)
    return h.hexdigest()


def test_l7_preset_blocks_equal_cli(tmp_path):
    """configs[3]'s shape at the preset block size (500 MB, fqzcomp5.c:4918):
    3 blocks of a 1.1 GB ONT file through the file path, equal to the
    reference's -7 -t1 output (its md5, recorded here by make_golden_l7.py)."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden_l7 as G
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "l7_ont.json")))
    src = str(tmp_path / "ont.fastq")
    assert G.make_input(src) == rec["in_bytes"]
    dst, back = str(tmp_path / "ont.fqz5"), str(tmp_path / "back.fastq")
    assert fqz5file.compress_file(src, dst, 7) == rec["out_bytes"]
    assert _md5(dst) == rec["out_md5"]
    os.unlink(src)
    fqz5file.decompress_file(dst, back)
    assert _md5(back) == rec["in_md5"]


def test_l9_paired_preset_blocks_equal_cli(tmp_path):
    """configs[4] at reduced size: two-file paired HiFi
    (load_seqs_interleaved, fqzcomp5.c:627-865) at -9 with the preset's 1 GB
    blocks (:4931), 2.28 GB in 3 blocks, through compress_file(src2=...):
    equal to the reference's -9 -t1 r1 r2 output (its md5, recorded by
    tests/golden/make_golden_l9_pairs.py), and decoded back to both files."""
    import sys
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden_l9_pairs as G
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "l9_pairs.json")))
    r1, r2 = str(tmp_path / "r1.fastq"), str(tmp_path / "r2.fastq")
    assert G.make_inputs(r1, r2) == (rec["r1_bytes"], rec["r2_bytes"])
    dst = str(tmp_path / "pairs.fqz5")
    assert fqz5file.compress_file(r1, dst, 9, src2=r2) == rec["out_bytes"]
    assert _md5(dst) == rec["out_md5"]
    os.unlink(r1)
    os.unlink(r2)
    b1, b2 = str(tmp_path / "b1.fastq"), str(tmp_path / "b2.fastq")
    fqz5file.decompress_file(dst, b1, dst2=b2)
    assert (_md5(b1), _md5(b2)) == (rec["r1_md5"], rec["r2_md5"])


def test_l5_illumina_file_equals_cli(tmp_path):
    """-5 on 1.54 GB of random-walk Illumina (15 preset
    blocks) through compress_file, the window sized from the level's
    footprint: equal to the reference's -5 -t1 output (md5 recorded by
    tests/golden/make_golden_l5.py), the arenas' device peak within the
    footprint the window is sized by (fqz5file.FOOTPRINT), and decoded
    back."""
    import sys
    from fqzcomp5_amd import lib
    sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
    import make_golden_l5 as G
    rec = json.load(open(os.path.join(ROOT, "tests", "golden", "l5_illumina.json")))
    src = str(tmp_path / "illumina.fastq")
    assert G.make_input(src) == rec["in_bytes"]
    dst, back = str(tmp_path / "illumina.fqz5"), str(tmp_path / "back.fastq")
    lib.arena_peak(reset=True)
    assert fqz5file.compress_file(src, dst, 5) == rec["out_bytes"]
    peak = lib.arena_peak()
    assert _md5(dst) == rec["out_md5"]
    assert peak <= fqz5file.FOOTPRINT[5] * rec["in_bytes"], peak
    os.unlink(src)
    fqz5file.decompress_file(dst, back)
    assert _md5(back) == rec["in_md5"]
