"""The read-once multi-rank window (fqz5file._next_window_ranks) on CPU
ranks (gloo), with the GPU record parse stood in for by a host FASTQ/FASTA
indexer of the same record table: every rank must see the one-process block
split, owners, per-block section sizes and FASTA flags, and gather exactly
the text of the blocks it needs, while reading about its share of the file.
(The GPU runs of the same path are tests/test_stream_gpu.py.)"""
import ctypes as C
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from fqzcomp5_amd import fqz5file, synth


def _py_index(text_d, at, n):
    """fqz5_fastq_index's record table for 4-line FASTQ or FASTA text:
    name / comment / seq / qual offsets and lengths, load_seqs_kseq sizes."""
    t = bytes(text_d[at:at + n].numpy())
    recs, rsz = [], []
    fasta = n > 0 and t[0:1] == b">"
    lines = t.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    offs, o = [], 0
    for ln in lines:
        offs.append(o)
        o += len(ln) + 1
    i = 0
    while i < len(lines):
        h = lines[i]
        sp = [k for k in range(1, len(h)) if h[k:k + 1] in (b" ", b"\t")]
        nl = (sp[0] if sp else len(h)) - 1
        cl = len(h) - nl - 2 if sp else 0
        if fasta:
            j = i + 1
            seq = b""
            while j < len(lines) and not lines[j].startswith(b">"):
                seq += lines[j]
                j += 1
            sl, ql, so, qo = len(seq), 0, offs[i + 1] if i + 1 < len(offs) else n, 0
            i_next = j
        else:
            sl, ql = len(lines[i + 1]), len(lines[i + 3])
            so, qo = offs[i + 1], offs[i + 3]
            i_next = i + 4
        recs.append((offs[i] + 1 + at, offs[i] + 2 + nl + at, so + at, qo + at, nl, cl, sl,
                     int(fasta)))
        rsz.append(nl + 1 + sl + ql)
        i = i_next
    w = C.sizeof(fqz5file.FastqRec)
    arr = (fqz5file.FastqRec * max(len(recs), 1))(*[fqz5file.FastqRec(*r) for r in recs])
    raw = np.frombuffer(bytes(arr), np.uint8)[:len(recs) * w].copy()
    return torch.from_numpy(raw), np.array(rsz, np.uint32), len(recs), fasta


class _FakeRun:
    def __init__(self, text, recs, ranges):
        self.text, self.ranges = text, ranges
        w = C.sizeof(fqz5file.FastqRec)
        u = recs.view(-1, w)[:, 32:44].contiguous().view(torch.int32).view(-1, 3).numpy()
        nsz = u[:, 0] + np.where(u[:, 1] > 0, u[:, 1] + 1, 0) + 1
        self.spans, self.blk_sec0 = [], []
        for a, b in ranges:
            self.blk_sec0.append(len(self.spans))
            self.spans.append((0, 0, int(nsz[a:b].sum())))
            self.spans.append((1, 0, int(u[a:b, 2].sum())))


def _fake_gather(text_d, recs, ranges, fasta, pairs):
    return _FakeRun(bytes(text_d.numpy()), recs, ranges)


def _rank(rank, world, port, args, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fqz5file._index_text = _py_index
    fqz5file._gather_ranges = _fake_gather
    try:
        paths, blk, wb = args
        files = [fqz5file._PosFile(p) for p in paths]
        at = [0] * len(files)
        fqz5file.H2D[0] = 0
        out = []
        while True:
            W = fqz5file._next_window_ranks(files, at, blk, wb, "cpu", dist.group.WORLD)
            if W is None:
                break
            need = [b for b in range(W.nb) if W.owner[b] == rank]
            run = W.gather(need)
            out.append(dict(first=[int(x) for x in W.first[:W.nb + 1]], owner=W.owner.tolist(),
                            nb=W.nb, fasta=W.fasta, nbytes=W.name_bytes, sbytes=W.seq_bytes,
                            nrec=W.nrec, need=need, text=run.text, pos=list(at)))
            W.advance()
        q.put((rank, out, fqz5file.H2D[0], None))
    except Exception as e:  # noqa: BLE001
        import traceback
        q.put((rank, None, 0, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(paths, blk, wb, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank, args=(r, world, port, (paths, blk, wb), q))
          for r in range(world)]
    for p in ps:
        p.start()
    res = sorted([q.get(timeout=300) for _ in range(world)], key=lambda x: x[0])
    for p in ps:
        p.join(timeout=60)
    for r in res:
        assert r[3] is None, r[3]
    return res


def _expect(paths, blk):
    """One process: the records of the whole input, its blocks."""
    so = fqz5file._load()
    texts = [open(p, "rb").read() for p in paths]
    idx = [_py_index(torch.frombuffer(bytearray(t), dtype=torch.uint8), 0, len(t)) for t in texts]
    if len(paths) == 1:
        first = fqz5file._blocks(so, idx[0][1], blk)
    else:
        k = idx[0][2]
        first = fqz5file._blocks(so, (idx[0][1][:k] + idx[1][1][:k]).astype(np.uint32), blk) * 2
    return texts, idx, [int(x) for x in first]


def _rec_bounds(text, idx):
    w = C.sizeof(fqz5file.FastqRec)
    v = idx[0].view(-1, w)[:, :8].contiguous().view(torch.int64).flatten().numpy()
    starts = (v - 1).tolist()
    return starts + [len(text)]


@pytest.mark.parametrize("kind", ["fastq", "fasta", "pairs"])
def test_rank_windows_match_one_process(tmp_path, kind):
    blk = 1_000_000
    if kind == "fastq":
        r = synth.illumina(26000, seed=3, with_names=True)
        p = str(tmp_path / "a.fq")
        synth.write_fastq(r, p)
        paths, wb = [p], 3_300_000
    elif kind == "fasta":
        r = synth.ont(300, seed=4, with_names=True)
        ends = np.cumsum(r.lens.astype(np.int64))
        txt = b"".join(
            b">%s\n%s\n" % (nm, b"\n".join(r.seq[a + k:min(a + k + 80, b)].tobytes()
                                           for k in range(0, b - a, 80)))
            for nm, a, b in zip(r.names, [0] + ends[:-1].tolist(), ends.tolist()))
        p = str(tmp_path / "a.fa")
        open(p, "wb").write(txt)
        paths, wb = [p], 2_500_000
    else:
        p1, p2 = str(tmp_path / "r1.fq"), str(tmp_path / "r2.fq")
        synth.write_fastq(synth.illumina(9000, seed=5, with_names=True), p1)
        synth.write_fastq(synth.novaseq(9000, seed=6, with_names=True), p2)
        paths, wb = [p1, p2], 2_200_000
    texts, idx, first = _expect(paths, blk)
    res = _run(paths, blk, wb)
    mul = 2 if kind == "pairs" else 1
    bounds = [_rec_bounds(t, i) for t, i in zip(texts, idx)]
    size = sum(len(t) for t in texts)
    # the windows' blocks, one after the other, are the one-process blocks
    for rank, out, h2d, _ in res:
        nbl = sum(w["nb"] for w in out)
        assert nbl == len(first) - 1, (rank, nbl, len(first) - 1)
        # every rank gathered the exact text of its blocks
        gb = 0
        for w in out:
            want = []
            for f, (t, bd) in enumerate(zip(texts, bounds)):
                pieces = []
                for b in w["need"]:
                    g0 = first[gb + b] // mul
                    g1 = first[gb + b + 1] // mul
                    pieces.append(t[bd[g0]:bd[g1]])
                want.append(b"".join(pieces))
            assert w["text"] == b"".join(want), (rank, kind)
            gb += w["nb"]
        # (small inputs: the trial's first three blocks are a large part of
        # them and every rank holds those; the GPU test bounds a 108 MB file
        # at 0.6 x)
        assert h2d <= (0.75 if kind == "fastq" else 1.2) * size, (rank, h2d, size)
    # and agree on the owners and sizes
    assert [w["owner"] for w in res[0][1]] == [w["owner"] for w in res[1][1]]
    assert [w["nbytes"] for w in res[0][1]] == [w["nbytes"] for w in res[1][1]]


def _rank_kind(rank, world, port, args, q):
    """The kind of each window _next_window_ranks returns (WRAPPED or a
    window of nb blocks), advancing over the 4-line windows."""
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fqz5file._index_text = _py_index
    fqz5file._gather_ranges = _fake_gather
    try:
        path, blk, wb = args
        files = [fqz5file._PosFile(path)]
        at = [0]
        kinds = []
        while True:
            W = fqz5file._next_window_ranks(files, at, blk, wb, "cpu", dist.group.WORLD)
            if W is None:
                break
            if W is fqz5file.WRAPPED:
                kinds.append(("wrapped", at[0]))
                break
            kinds.append(("four", W.nb))
            W.advance()
        q.put((rank, kinds, 0, None))
    except Exception:  # noqa: BLE001
        import traceback
        q.put((rank, None, 0, traceback.format_exc()))
    finally:
        dist.destroy_process_group()


def test_rank_windows_detect_wrapped(tmp_path):
    """a wrapped FASTQ (kseq.h:194-216) cannot be split
    by the 4-line count; every rank must see WRAPPED for the first window
    that holds wrapped records, at the same file offset, after the 4-line
    windows before it (the file path then reads those windows whole,
    fqz5file._encode_stream; its bytes: tests/test_stream_gpu.py)."""
    from wrapped_cases import illumina70
    four = synth.illumina(9000, seed=3, with_names=True)
    head = synth.fastq_chunk(four, 0, four.num_records).tobytes()
    p = str(tmp_path / "w.fq")
    open(p, "wb").write(head + illumina70())
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_kind, args=(r, 2, port, (p, 1_000_000, 1_500_000), q))
          for r in range(2)]
    for x in ps:
        x.start()
    res = sorted([q.get(timeout=300) for _ in range(2)], key=lambda x: x[0])
    for x in ps:
        x.join(timeout=60)
    assert all(r[3] is None for r in res), res
    k0, k1 = res[0][1], res[1][1]
    assert k0 == k1
    assert k0[-1][0] == "wrapped" and any(k == "four" for k, _ in k0[:-1]), k0
    # the wrapped window starts at a record boundary inside the 4-line head
    assert 0 < k0[-1][1] <= len(head)
    assert head[k0[-1][1]:k0[-1][1] + 1] == b"@"
