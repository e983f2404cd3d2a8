"""bench.py's multi-rank plumbing on CPU (gloo, world size 2): every rank runs
its own replica, the job time is the max over ranks, value is whole-job."""
import os
import socket

import torch
import torch.multiprocessing as mp

import bench


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    w, r, _, dev = bench.dist_setup()
    assert (w, r) == (world, rank)
    bench.barrier(w)
    dt = bench.max_over_ranks(0.5 + rank, w, dev)          # rank 1 is the slow one
    tps, audio = bench.throughput(dt, batch=2, steps=10, world=w)
    out[rank] = (dt, tps, audio)
    torch.distributed.destroy_process_group()


def test_two_rank_max_and_weak_scaling():
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_worker, args=(2, port, out), nprocs=2, join=True)
        res = dict(out)
    assert res[0] == res[1]
    dt, tps, audio = res[0]
    assert dt == 1.5
    assert abs(tps - 2 * 10 * 2 / 1.5) < 1e-9
    assert abs(audio - tps * 3200 / 24000) < 1e-9


def test_single_rank_defaults():
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK"):
        os.environ.pop(k, None)
    w, r, loc, dev = bench.dist_setup()
    assert (w, r, loc) == (1, 0, 0)
    assert bench.max_over_ranks(2.0, w, dev) == 2.0
