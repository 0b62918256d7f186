"""CPU, world_size 2: the multi-process path of bench.py without a GPU.

bench.py runs one process per GPU (torchrun).  Its N>1 pieces are exercised here on CPU:
  - exchange_uid: rank 0 publishes the RCCL unique id through a node-local file, the other ranks poll for it;
  - timed_steps: barrier + K steps + barrier + max over ranks (the contract's timed region), driven through a gloo
    control plane that stands in for the RCCL all-reduce of the shared context (same barrier()/max() interface);
  - the weak-scaling aggregation: value = all ranks' frames / the max-over-ranks time.
The RCCL transport itself needs GPUs (tests/test_gpu_stream_multi.py covers the single-rank communicator and the
receive-side blob layout).  The weight-blob layout every rank computes from the GGUF headers before the broadcast
(q3t_plan_weight_layout: the same allocation sequence, host only) is compared across two gloo ranks, together with the
size check comm_bcast_arenas runs (identical files pass, different files fail on every rank).
"""
import os
import sys
import time

import numpy as np
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


def _layout_worker(rank, world, port, paths, q):
    """one rank of a shared start-up, host side: lay out the weight blob from the GGUF headers (q3t_plan_weight_layout,
    the allocation sequence q3t_ctx_create_shared runs before the broadcast), then the checks across ranks over gloo:
    comm_bcast_arenas' size all-reduce (max of used and of -used must agree) and the whole offset vector"""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    sys.path.insert(0, os.path.join(REPO, "qwen3-tts-jetson_amd"))
    import torch
    import torch.distributed as dist
    import q3t
    try:
        off, used = q3t.plan_weight_layout(paths[rank])
        dist.init_process_group("gloo", rank=rank, world_size=world)
        v = torch.tensor([float(used), -float(used)], dtype=torch.float64)
        dist.all_reduce(v, op=dist.ReduceOp.MAX)
        sizes_agree = v[0].item() == -v[1].item()
        n = torch.tensor([len(off)], dtype=torch.int64)
        ns = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(ns, n)
        same = len({int(x.item()) for x in ns}) == 1
        if same:
            t = torch.from_numpy(off.astype(np.int64))
            ts = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(ts, t)
            same = all(torch.equal(ts[0], x) for x in ts)
        q.put((rank, used, len(off), bool(sizes_agree), bool(same), None))
        dist.destroy_process_group()
    except Exception as e:  # surface the failure in the parent
        q.put((rank, None, None, None, None, repr(e)))


def _run_layout(paths):
    import multiprocessing as mp
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_layout_worker, args=(r, len(paths), port, paths, q)) for r in range(len(paths))]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=180) for _ in procs)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for r in res:
        assert r[5] is None, r
    return res



def test_weight_layout_identical_across_ranks_world2():
    """every rank of a shared context lays out the same weight blob from the same GGUF headers: identical offsets and
    sizes (the precondition of the RCCL broadcast, whose receive side never reads tensor bytes)"""
    from q3t_testutil import synth_dir
    tts, _ = synth_dir("full")
    res = _run_layout([tts, tts])
    (_, u0, n0, ok0, same0, _), (_, u1, n1, ok1, same1, _) = res
    assert u0 == u1 > 0 and n0 == n1 > 100
    assert ok0 and ok1 and same0 and same1


def test_weight_layout_mismatch_detected_world2():
    """ranks handed different model files: the size check comm_bcast_arenas runs before broadcasting fails on every rank"""
    from q3t_testutil import synth_dir
    tts_full, _ = synth_dir("full")
    tts_tiny, _ = synth_dir("tiny")
    res = _run_layout([tts_full, tts_tiny])
    (_, u0, _, ok0, same0, _), (_, u1, _, ok1, same1, _) = res
    assert u0 != u1
    assert not ok0 and not ok1 and not same0 and not same1
