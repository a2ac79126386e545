"""The only cross-rank step of the section coder: every rank
all-gathers the candidate sizes of its sections, then replays the -t1 trial
state over the whole file.  Two gloo ranks on the CPU must reach exactly
the method choices of one process replaying the concatenated rows."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

from fqzcomp5_amd import sections as S


def _rows(rank: int, nblocks: int):
    rng = np.random.default_rng(100 + rank)
    ids, ins, sizes = [], [], []
    for _ in range(nblocks):
        for sec in (S.SEC_SEQ, S.SEC_QUAL):
            n = int(rng.integers(10_000, 100_000))
            row = np.zeros(S.M_LAST, np.uint32)
            # candidate sizes for every method bit; 0 = not tried
            row[1:10] = rng.integers(n // 8, n // 2, 9)
            ids.append(sec)
            ins.append(n)
            sizes.append(row)
    return np.array(ids, np.int32), np.array(ins, np.uint32), np.stack(sizes)


def _worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    ids, ins, sizes = _rows(rank, 5 + rank)
    g_sizes, g_ins, g_ids, off = S.exchange_sizes(sizes, ins, ids)
    st = S.new_state()
    meth = S.trial_replay(g_ids, g_ins, g_sizes, S.masks(3), st)
    q.put((rank, off, meth[off:off + len(ids)].tolist(), g_ids.tolist()))
    dist.destroy_process_group()


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_two_ranks_match_single_process_replay():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    got = dict()
    for _ in range(world):
        r, off, meth, gids = q.get(timeout=120)
        got[r] = (off, meth, gids)
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    # single process: rank-major concatenation = file order
    parts = [_rows(r, 5 + r) for r in range(world)]
    ids = np.concatenate([p[0] for p in parts])
    ins = np.concatenate([p[1] for p in parts])
    sizes = np.concatenate([p[2] for p in parts])
    ref = S.trial_replay(ids, ins, sizes, S.masks(3), S.new_state()).tolist()
    assert got[0][0] == 0 and got[1][0] == len(parts[0][0])
    assert got[0][2] == ids.tolist() == got[1][2]
    assert got[0][1] + got[1][1] == ref


def test_schedule_matches_replay():
    """The size-free schedule names exactly the sections that try every
    method in a full replay (trial and re-trial blocks: 3 per 100)."""
    rng = np.random.default_rng(9)
    ids = np.array([S.SEC_SEQ, S.SEC_QUAL] * 230, np.int32)
    ins = rng.integers(10_000, 100_000, len(ids)).astype(np.uint32)
    sizes = np.full((len(ids), S.M_LAST), 0xFFFFFFFF, np.uint32)
    sizes[:, 1:10] = rng.integers(1_000, 50_000, (len(ids), 9))
    av = S.masks(3)
    sched = S.trial_schedule(ids, av, S.new_state())
    tried = np.zeros(len(ids), np.uint32)
    S.trial_replay(ids, ins, sizes, av, S.new_state(), tried)
    multi = np.array([bin(int(t)).count("1") > 1 for t in tried])
    assert (sched[multi] == tried[multi]).all()
    assert (sched[~multi] == 0).all()
    assert multi.sum() == 2 * 3 * 3        # blocks 1-3, 104-106, 207-209 per section
