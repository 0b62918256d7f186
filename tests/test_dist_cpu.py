"""CPU, world_size 2: the multi-process path of bench.py without a GPU.

bench.py runs one process per GPU (torchrun).  Its N>1 pieces are exercised here on CPU:
  - exchange_uid: rank 0 publishes the RCCL unique id through a node-local file, the other ranks poll for it;
  - timed_steps: barrier + K steps + barrier + max over ranks (the contract's timed region), driven through a gloo
    control plane that stands in for the RCCL all-reduce of the shared context (same barrier()/max() interface);
  - the weak-scaling aggregation: value = all ranks' frames / the max-over-ranks time.
The RCCL transport itself needs GPUs (tests/test_gpu_stream_multi.py covers the single-rank communicator and the
receive-side blob layout).
"""
import os
import sys
import time

import pytest

from q3t_testutil import REPO

sys.path.insert(0, REPO)


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


class GlooCtrl:
    def __init__(self, dist):
        self.dist = dist

    def barrier(self):
        self.dist.barrier()

    def max(self, v):
        import torch
        t = torch.tensor([v], dtype=torch.float64)
        self.dist.all_reduce(t, op=self.dist.ReduceOp.MAX)
        return float(t.item())


def _worker(rank, world, port, uid_dir, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      Q3T_UID_DIR=uid_dir)
    import torch.distributed as dist
    import bench
    try:
        uid = bench.exchange_uid(rank, (lambda: bytes(range(128))) if rank == 0 else None, timeout=60)
        dist.init_process_group("gloo", rank=rank, world_size=world)
        ctrl = GlooCtrl(dist)
        frames_per_step = 7
        done = []

        def step(k):
            time.sleep(0.05 * (rank + 1))   # rank 1 is the slow one
            done.append(frames_per_step)

        elapsed = bench.timed_steps(ctrl, lambda: None, step, 3)
        total = world * frames_per_step * 3
        if rank == 0:
            bench.release_uid()
        q.put((rank, uid, elapsed, total / elapsed, len(done)))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, None, repr(e), None, None))


def test_bench_multiprocess_plumbing_world2(tmp_path):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, str(tmp_path), q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    (r0, uid0, el0, v0, n0), (r1, uid1, el1, v1, n1) = res
    assert uid0 == uid1 == bytes(range(128)), (uid0, uid1, el0, el1)
    # max over ranks: both ranks report the slow rank's time (3 x 0.1 s), hence the same aggregate value
    assert el0 == el1 >= 0.3
    assert v0 == v1 == pytest.approx(2 * 7 * 3 / el0)
    assert n0 == n1 == 3
    assert not any(f.startswith("q3t_rccl_uid") for f in os.listdir(tmp_path))


def test_uid_exchange_times_out_without_rank0(tmp_path, monkeypatch):
    import bench
    monkeypatch.setenv("Q3T_UID_DIR", str(tmp_path))
    monkeypatch.setenv("MASTER_PORT", "1")
    with pytest.raises(RuntimeError, match="no RCCL id"):
        bench.exchange_uid(1, None, timeout=0.2)
