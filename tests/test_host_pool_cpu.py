"""The library's host thread pools are sized per rank:
host::threads() = the process's CPU affinity mask divided by
$LOCAL_WORLD_SIZE (torch.distributed.run's ranks on this node), capped by
$OMP_NUM_THREADS and at 16; $FQZ5_HOST_THREADS overrides.  Run in child
processes (the value is fixed at first use) without touching the GPU."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROBE = r"""
import ctypes, os, sys
cpus = [int(x) for x in sys.argv[1].split(",")]
os.sched_setaffinity(0, cpus)
so = ctypes.CDLL(os.path.join(sys.argv[2], "fqzcomp5_amd", "libfqz5_mi355x.so"))
print(so.fqz5_host_threads())
"""


def _threads(cpus, **env):
    e = {k: v for k, v in os.environ.items()
         if k not in ("LOCAL_WORLD_SIZE", "OMP_NUM_THREADS", "FQZ5_HOST_THREADS")}
    e.update({k: str(v) for k, v in env.items()})
    r = subprocess.run([sys.executable, "-c", PROBE, ",".join(map(str, cpus)), ROOT],
                       capture_output=True, text=True, env=e, timeout=120, check=True)
    return int(r.stdout.strip().splitlines()[-1])


avail = sorted(os.sched_getaffinity(0))
need8 = pytest.mark.skipif(len(avail) < 8, reason="needs 8 usable CPUs")


@need8
def test_pool_is_the_ranks_share():
    cpus = avail[:8]
    assert _threads(cpus) == 8
    # eight ranks on this node: each gets at most cores / 8
    assert _threads(cpus, LOCAL_WORLD_SIZE=8) == 1
    assert _threads(cpus, LOCAL_WORLD_SIZE=2) == 4
    assert _threads(cpus, LOCAL_WORLD_SIZE=3) == 2


@need8
def test_pool_follows_affinity_not_hardware():
    # hardware_concurrency() would say every CPU of the machine
    assert _threads(avail[:3]) == 3
    assert _threads(avail[:1], LOCAL_WORLD_SIZE=4) == 1


@need8
def test_pool_caps():
    assert _threads(avail[:8], OMP_NUM_THREADS=2) == 2
    assert _threads(avail[:8], FQZ5_HOST_THREADS=5, LOCAL_WORLD_SIZE=8) == 5
