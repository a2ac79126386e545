"""One rank fails mid-window: every rank raises, none waits for the process
group's timeout (sections.xchg / ranks_fail_together).

gloo ranks on the CPU run several windows of sections.encode_window with
the GPU calls replaced by test_window_cpu's deterministic fake codec, inside
ranks_fail_together with a final barrier, as fqz5file.compress_file runs
them.  One rank's fake commit raises in its third window, after that
window's size exchange and before the block-size exchange that follows.
Every process must exit non-zero well within 60 s: the failing rank with its
own error, the others with PeerError naming it."""
import os
import time

import numpy as np
import pytest
import torch.multiprocessing as mp

from fqzcomp5_amd import sections as S
from test_window_cpu import _Fake, _free_port, _layout


def _windows(world, rank, fail_rank, fail_window, level=5, nblocks=4, windows=5):
    import torch.distributed as dist
    group = dist.group.WORLD
    st = S.new_state()
    fake = _Fake()
    calls = [0]
    commit = fake.sections_commit

    def failing_commit(secs, meth):
        calls[0] += 1
        if rank == fail_rank and calls[0] == fail_window + 1:
            raise RuntimeError(f"injected failure on rank {rank}")
        return commit(secs, meth)
    S.sections_try, S.sections_commit = fake.sections_try, failing_commit
    S.sections_try_bounds = fake.sections_try_bounds
    with S.ranks_fail_together(group):
        for w in range(windows):
            ids, ins = _layout(nblocks, level)
            secs = [S.Section(None, None, int(ins[i]), 0, 0, int(ids[i]), None, None, i, None)
                    for i in range(len(ids))]
            owner = np.repeat((np.arange(nblocks) * world) // nblocks, 3)
            S.encode_window(secs, ids, ins, owner, S.masks(level, full=True), st, group)
            # the per-window block-size exchange of fqz5file._code_window
            S.xchg([w, rank], group)
        S.barrier(group)


def _worker(rank, world, port, q, fail_rank, fail_window):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _windows(world, rank, fail_rank, fail_window)
        q.put((rank, "ok", ""))
        code = 0
    except Exception as e:          # noqa: BLE001 (the test reads the type)
        q.put((rank, type(e).__name__, str(e)[:200]))
        code = 1
    raise SystemExit(code)


@pytest.mark.parametrize("world,fail_rank", [(2, 1), (3, 0), (3, 2)])
def test_one_rank_fails_all_exit(world, fail_rank):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    t0 = time.time()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q, fail_rank, 2))
          for r in range(world)]
    for p in ps:
        p.start()
    got = {}
    try:
        for _ in range(world):
            r, kind, msg = q.get(timeout=60)
            got[r] = (kind, msg)
        for p in ps:
            p.join(timeout=30)
    finally:
        for p in ps:
            if p.is_alive():
                p.kill()
    assert time.time() - t0 < 60
    assert all(p.exitcode == 1 for p in ps), [p.exitcode for p in ps]
    assert got[fail_rank][0] == "RuntimeError"
    for r in range(world):
        if r != fail_rank:
            assert got[r][0] == "PeerError" and f"rank {fail_rank}" in got[r][1], got[r]


def test_no_failure_all_ok():
    """The same windows with nobody failing: every rank returns."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, 2, port, q, -1, 2)) for r in range(2)]
    for p in ps:
        p.start()
    got = [q.get(timeout=60) for _ in range(2)]
    for p in ps:
        p.join(timeout=30)
    assert sorted(k for _, k, _ in got) == ["ok", "ok"]
    assert all(p.exitcode == 0 for p in ps)
