"""Host logic of the streaming / multi-GPU file path (fqzcomp5_amd/fqz5file.py,
sections.encode_window), on the CPU.

* encode_window over two gloo ranks, with the GPU calls (sections_try /
  sections_commit) replaced by a deterministic fake codec: the methods
  chosen equal a single process's, every rank commits only its own sections,
  the trial sections' work candidates (fqz, sequence models, LZP3) are split
  over the ranks by method and each is tried exactly once, and the collective
  is the only exchange (fqzcomp5.c:1899-1958 trial, :3108-3115 offsets).
* the window cut rule (_complete_records) on FASTA text.
* the .fqz5 reader's checks: truncated files and blocks whose sizes disagree
  are refused on the host, before any device work.
"""
import os
import socket
import struct
import subprocess
import zlib

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from fqzcomp5_amd import fqz5file
from fqzcomp5_amd import sections as S

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CLI = os.path.join(ROOT, "oracle", "_ref", "fqzcomp5")


def _layout(nblocks: int, level: int):
    ids, ins = [], []
    rng = np.random.default_rng(7)
    for _ in range(nblocks):
        for sec in (S.SEC_NAME, S.SEC_SEQ, S.SEC_QUAL):
            ids.append(sec)
            ins.append(int(rng.integers(50_000, 100_000)))
    return np.array(ids, np.int32), np.array(ins, np.uint32)


def _fake_size(i: int, m: int, n: int) -> int:
    """A deterministic candidate size: any method may win anywhere."""
    h = (i * 2654435761 + m * 40503 + 17) & 0xFFFFFFFF
    return n // 4 + h % (n // 3)


class _Fake:
    """Stands in for the GPU calls: records what was tried / committed."""

    def __init__(self, width: int = 0):
        self.tried, self.committed, self.sess = [], [], None
        self.width = width      # bounds tries: fqz / sequence-model interval width

    def sections_try_bounds(self, secs, masks):
        lo = self.sections_try(secs, masks)
        hi = lo.copy()
        iv = [m for m in range(S.M_LAST) if (1 << m) & (S.FQZ_MASK | S.SEQ_MASK)]
        sel = lo[:, iv] != 0xFFFFFFFF
        v = lo[:, iv].astype(np.int64)
        lo[:, iv] = np.where(sel, np.maximum(v - self.width, 1), v).astype(np.uint32)
        hi[:, iv] = np.where(sel, v + self.width, v).astype(np.uint32)
        return lo, hi

    def sections_try(self, secs, masks):
        out = np.full((len(secs), S.M_LAST), 0xFFFFFFFF, np.uint32)
        for k, (s, m) in enumerate(zip(secs, masks)):
            for b in range(S.M_LAST):
                if (int(m) >> b) & 1:
                    out[k, b] = _fake_size(s.nrec, b, s.in_size)
                    self.tried.append((s.nrec, b))
        self.sess = [s.nrec for s in secs]
        return out

    def sections_commit(self, secs, meth):
        assert [s.nrec for s in secs] == self.sess, "commit without its try"
        res = []
        for s, m in zip(secs, meth):
            r = S.SectionResult()
            r.method, r.status = int(m), 0 if m > 0 else -1
            if m > 0:
                self.committed.append((s.nrec, int(m)))
            res.append(r)
        self.sess = None
        return res


def _run(world: int, rank: int, nblocks: int, level: int, bounded: bool, width: int = 0,
         bounds: bool = True):
    ids, ins = _layout(nblocks, level)
    n = len(ids)
    secs = []
    for i in range(n):   # Section.nrec carries the section index for the fake
        secs.append(S.Section(None, None, int(ins[i]), 0, 0, int(ids[i]), None, None, i, None))
    owner = np.repeat((np.arange(nblocks) * world) // nblocks, 3)
    fake = _Fake(width)
    S.sections_try, S.sections_commit = fake.sections_try, fake.sections_commit
    S.sections_try_bounds = fake.sections_try_bounds
    st = S.new_state()
    group = None
    if world > 1:
        import torch.distributed as dist
        group = dist.group.WORLD
    res, meth, sizes = S.encode_window(secs, ids, ins, owner, S.masks(level, full=True), st,
                                       group, bounded=bounded, bounds=bounds)
    return dict(meth=meth.tolist(), tried=fake.tried, committed=fake.committed,
                owned=[i for i in range(n) if res[i] is not None],
                decided=S.last_bounds_decided)


def _worker(rank, world, port, q, args):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank, _run(world, rank, *args)))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@pytest.mark.parametrize("level,nblocks,bounded", [(5, 6, False), (7, 5, True), (9, 4, True)])
def test_encode_window_two_ranks(level, nblocks, bounded):
    single = _run(1, 0, nblocks, level, bounded)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, (nblocks, level, bounded)))
          for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        r, out = q.get(timeout=120)
        got[r] = out
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # the same choices as one process
    assert got[0]["meth"] == got[1]["meth"] == single["meth"]
    # every section committed once, by its owner, with its method
    owner = (np.arange(nblocks) * world) // nblocks
    for r in range(world):
        assert all(owner[i // 3] == r for i in got[r]["owned"])
        assert all(owner[i // 3] == r for i, _ in got[r]["committed"])
    assert sorted(got[0]["committed"] + got[1]["committed"]) == sorted(single["committed"])
    # the trial's work candidates: split over the ranks, each tried once
    work = lambda t: sorted((i, m) for i, m in t if (1 << m) & S.WORK_MASK)
    w0, w1, ws = work(got[0]["tried"]), work(got[1]["tried"]), work(single["tried"])
    assert w0 and w1, "both ranks run work candidates"
    assert not set(w0) & set(w1)
    assert sorted(w0 + w1) == ws
    # and all of block 0's (the first trial block) are not on one rank
    assert {m for i, m in w0 if i < 3} and {m for i, m in w1 if i < 3}


def test_work_share_partitions_methods():
    ms = [S.FQZ0, S.FQZ1, S.FQZ2, S.FQZ3, S.FQZ4, S.SEQ10, S.LZP3]
    for world in (1, 2, 3, 8):
        shares = [S.work_share(ms, world, r) for r in range(world)]
        assert sum(bin(x).count("1") for x in shares) == len(ms)
        acc = 0
        for x in shares:
            assert not acc & x
            acc |= x
        assert acc == sum(1 << m for m in ms)


def test_window_cut_rules():
    """FASTA on the host (the FASTQ rule runs on the GPU:
    test_wrapped_fastq_gpu.py::test_record_ends)."""
    fa_txt = b">x\nACGT\nAC\n>y 1\nGG\n\n>z\nT"
    t = torch.frombuffer(bytearray(fa_txt), dtype=torch.uint8)
    ends, fa = fqz5file._complete_records(t, len(fa_txt), False)
    assert fa and ends == [fa_txt.index(b">y"), fa_txt.index(b">z")]
    ends, _ = fqz5file._complete_records(t, len(fa_txt), True)
    assert ends[-1] == len(fa_txt)


@pytest.fixture(scope="module")
def cli_file(tmp_path_factory):
    if not os.path.exists(CLI):
        pytest.skip("reference CLI not built")
    from fqzcomp5_amd import synth
    d = tmp_path_factory.mktemp("blk")
    src, out = str(d / "in.fastq"), str(d / "o.fqz5")
    synth.write_fastq(synth.illumina(8000, seed=4, with_names=True), src)
    subprocess.run([CLI, "-3", "-t1", "-b", "500k", src, out], check=True, capture_output=True)
    return open(out, "rb").read()


def test_block_text_sizes_from_headers(tmp_path):
    """decompress_file's multi-rank offsets: each block's FASTQ text size from
    its headers alone equals the text the block came from (and with the
    name repeated on the '+' line, that plus the names)."""
    if not os.path.exists(CLI):
        pytest.skip("reference CLI not built")
    from fqzcomp5_amd import synth
    r = synth.illumina(9000, seed=12, with_names=True)
    src, out = str(tmp_path / "in.fastq"), str(tmp_path / "o.fqz5")
    synth.write_fastq(r, src)
    subprocess.run([CLI, "-5", "-t1", "-b", "400k", src, out], check=True, capture_output=True)
    text = open(src, "rb").read()
    with open(out, "rb") as f:
        ranges = fqz5file._file_blocks(f, os.path.getsize(out))
        assert len(ranges) > 2
        sizes = [fqz5file._block_text_size(f, s, e, False) for s, e in ranges]
        plus = [fqz5file._block_text_size(f, s, e, True) for s, e in ranges]
    assert sum(sizes) == len(text)
    names = sum(len(r.name(i).split(b" ")[0]) + (len(r.name(i)) - len(r.name(i).split(b" ")[0]))
                for i in range(r.num_records))
    assert sum(plus) == len(text) + names


def test_truncated_file_refused(cli_file):
    data = cli_file
    ranges = fqz5file._blocks_of(data)
    assert len(ranges) > 1 and [f["seq_ulen"] == f["qual_ulen"] for f in
                                fqz5file.check_blocks(data)] == [True] * len(ranges)
    idx = struct.unpack_from("<Q", data, 8)[0]
    with pytest.raises(ValueError):      # the index offset past the end
        fqz5file._blocks_of(data[:idx - 1])
    cut = bytearray(data[:ranges[1][0] + 100])
    cut[8:16] = struct.pack("<Q", 0)     # no index: the block walk runs off the end
    with pytest.raises(ValueError):
        fqz5file._blocks_of(bytes(cut))


def test_mismatched_sizes_refused(cli_file):
    data = bytearray(cli_file)
    s, e = fqz5file._blocks_of(data)[0]
    f = fqz5file.block_fields(data, s, e)
    # walk to the quality section header and grow its u_len by one, then
    # fix the CRC so that only the size check can catch it
    p = s + 12
    nu, _, nc = struct.unpack_from("<IBI", data, p)
    p += 9 + nc
    nb = data[p]
    p += 1 + (nb if nb else 4 + struct.unpack_from("<I", data, p + 1)[0])
    _, su, sc = struct.unpack_from("<BII", data, p)
    p += 9 + sc
    st, qu, qc = struct.unpack_from("<BII", data, p)
    assert qu == su == f["seq_ulen"]
    struct.pack_into("<BII", data, p, st, qu + 1, qc)
    struct.pack_into("<I", data, s + 8, zlib.crc32(bytes(data[s + 12:e])))
    with pytest.raises(ValueError, match="quality and sequence"):
        fqz5file.check_blocks(bytes(data))


def test_lengths_header_count_not_trusted(cli_file):
    """The fixed-length header [nb][varint] is walked by the varint's own
    bytes, as decode_block reads it (fqzcomp5.c:2384-2395), not by nb: a
    CRC-valid block whose nb lies parses to the same sections, and a quality
    u_len past the bases behind that lie is refused (the decoders size their
    outputs from these fields)."""
    data = bytearray(cli_file)
    s, e = fqz5file._blocks_of(data)[0]
    f0 = fqz5file.block_fields(data, s, e)
    p = s + 12
    nu, _, nc = struct.unpack_from("<IBI", data, p)
    p += 9 + nc
    assert data[p] > 0                      # fixed-length block
    vl = 1
    while data[p + vl] & 0x80:
        vl += 1
    data[p] = 5                             # claims 5 bytes, the varint is vl
    crc = lambda: struct.pack_into("<I", data, s + 8, zlib.crc32(bytes(data[s + 12:e])))
    crc()
    f = fqz5file.block_fields(bytes(data), s, e)
    assert (f["seq_ulen"], f["qual_ulen"], f["nrec"]) == (f0["seq_ulen"], f0["qual_ulen"], f0["nrec"])
    q = p + 1 + vl
    _, su, sc = struct.unpack_from("<BII", data, q)
    q += 9 + sc
    st, qu, qc = struct.unpack_from("<BII", data, q)
    struct.pack_into("<BII", data, q, st, qu + 4096, qc)
    crc()
    with pytest.raises(ValueError, match="quality and sequence"):
        fqz5file.block_fields(bytes(data), s, e)


def test_lengths_sum_checked(cli_file):
    """Record lengths that do not cover the bases are refused (a CRC-valid
    block with the fixed length one larger)."""
    data = bytearray(cli_file)
    s, e = fqz5file._blocks_of(data)[0]
    p = s + 12
    nu, _, nc = struct.unpack_from("<IBI", data, p)
    p += 9 + nc
    assert data[p] > 0
    data[p + data[p]] += 1                  # the last varint byte: length + 1
    struct.pack_into("<I", data, s + 8, zlib.crc32(bytes(data[s + 12:e])))
    with pytest.raises(ValueError, match="lengths do not sum"):
        fqz5file.block_fields(bytes(data), s, e)


@pytest.mark.parametrize("width", [0, 5, 20000])
def test_bounded_intervals_choose_as_exact_sizes(width):
    """The -7 bounded window with interval tries (every fqz / sequence-model
    size known to +-width only) picks the methods of exact sizes: decided
    from the intervals when they separate the candidates, else the open
    candidates are coded exactly and the trial replayed (width 20000: the
    intervals overlap)."""
    exact = _run(1, 0, 5, 7, True, bounds=False)
    got = _run(1, 0, 5, 7, True, width=width)
    assert got["meth"] == exact["meth"]
    assert sorted(got["committed"]) == sorted(exact["committed"])
    assert got["decided"]
    work = lambda t: [x for x in t if (1 << x[1]) & S.WORK_MASK]
    if width == 0:       # every work candidate tried once
        assert sorted(work(got["tried"])) == sorted(set(work(got["tried"])))
    if width == 20000:   # some again, exactly
        assert len(work(got["tried"])) > len(set(work(got["tried"])))


def test_bounded_intervals_two_ranks_refine():
    """Over two ranks the candidates that overlapping intervals leave open
    are coded exactly, split over the ranks; the choices equal one process's
    exact ones."""
    exact = _run(1, 0, 5, 7, True, bounds=False)
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, (5, 7, True, 20000)))
          for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    for _ in range(world):
        r, out = q.get(timeout=120)
        got[r] = out
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert got[0]["meth"] == got[1]["meth"] == exact["meth"]
    assert got[0]["decided"] and got[1]["decided"]
    # some work candidates were coded twice over the ranks (interval, then
    # exact), each exact one on one rank only
    work = lambda t: [x for x in t if (1 << x[1]) & S.WORK_MASK]
    w0, w1 = work(got[0]["tried"]), work(got[1]["tried"])
    assert len(w0) + len(w1) > len(set(w0) | set(w1))


def test_refine_session_counts_late_sections():
    """a reused refinement session commits every section at once
    (no chunks), so refine_session refuses when the sections the commit codes
    late would take the session past its budget, or the inputs past one
    commit chunk; it returns False before any device work."""
    nsec = 12
    ids = np.array([S.SEC_NAME, S.SEC_SEQ, S.SEC_QUAL] * (nsec // 3), np.int32)
    ins = np.full(nsec, 1_000_000, np.uint32)
    sched = np.zeros(nsec, np.uint32)
    secs = [None] * nsec
    lo = np.zeros((nsec, S.M_LAST), np.uint32)
    hi = lo.copy()
    pairs = [(2, S.FQZ1)]
    # the open pair and its kind's sections alone fit, the late ones do not
    assert not S.refine_session(secs, ids, sched, lo, hi, pairs, ins, chunk_bytes=1_500_000)
    # inputs past one commit chunk
    assert not S.refine_session(secs, ids, sched, lo, hi, pairs, ins, chunk_bytes=10 ** 9,
                                commit_bytes=nsec * 1_000_000 - 1)


def test_rank_window_record_ends(tmp_path):
    """The multi-rank window's host helpers: the end of a record read on from
    its start (FASTQ: 4 lines, FASTA: up to the next '>' line, the file end
    closing the last one) and the merge of adjacent byte ranges."""
    t = b"@r1 c\nACGT\n+\nIIII\n@r2\nAC\n+\n@I\n@r3\nG\n+\nI"
    p = tmp_path / "a.fq"
    p.write_bytes(t)
    f = fqz5file._PosFile(str(p))
    assert [fqz5file._record_end(f, t.index(x), False) for x in (b"@r1", b"@r2", b"@r3")] == \
        [t.index(b"@r2"), t.index(b"@r3"), len(t)]
    f.close()
    u = b">a\nACG\nTT\n>b\nGG\n>c\nA\n" + b"C" * 200000 + b"\n>d\nA\n"
    q = tmp_path / "a.fa"
    q.write_bytes(u)
    g = fqz5file._PosFile(str(q))
    assert [fqz5file._record_end(g, u.index(x), True) for x in (b">a", b">b", b">c", b">d")] == \
        [u.index(b">b"), u.index(b">c"), u.index(b">d"), len(u)]
    g.close()
    assert fqz5file._merge([(0, 5), (5, 9), (12, 14), (14, 20)]) == [(0, 9), (12, 20)]


def test_window_sized_from_footprint():
    """The encode window from the level's device footprint: 0.8 x HBM per
    rank at FOOTPRINT bytes per input byte, at most 8 GB per rank, and never
    fewer than two blocks per rank and one over."""
    hbm = 288 << 30
    w5 = fqz5file.window_bytes_for(5, 100_000_000, 1, hbm)
    assert w5 * fqz5file.FOOTPRINT[5] <= 0.8 * hbm and w5 >= 3_000_000_000
    assert fqz5file.window_bytes_for(5, 100_000_000, 4, hbm) == 4 * w5
    assert fqz5file.window_bytes_for(1, 1_000_000, 1, hbm) == 8_000_000_000
    assert fqz5file.window_bytes_for(9, 1_000_000_000, 8, 8 << 30) == 17_000_000_000
