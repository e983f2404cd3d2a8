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


def _run_bench(args, env_extra=None, timeout=240):
    import json
    import subprocess
    import sys
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_PORT")}
    env.update(env_extra or {})
    env["CUDA_VISIBLE_DEVICES"] = ""         # CPU host path (gloo) even where a GPU is visible
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py")] + args, env=env, capture_output=True,
                       text=True, timeout=timeout)
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    return p.returncode, (json.loads(lines[-1]) if lines else None), p.stderr


def test_bench_gpus_flag_launches_ranks():
    """`python bench.py --gpus 2` starts two ranks itself (torch.distributed.run
    child on 127.0.0.1) and reports n_gpus 2; the job time is the slowest
    rank's (rank 1 sleeps 2 ms per step)."""
    rc, line, err = _run_bench(["--gpus", "2", "--plumbing", "--steps", "20", "--batch", "3"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 2 and line["backend"] == "gloo"
    assert line["ms_per_step"] >= 2.0
    assert abs(line["value"] - 3 * 2 * 3200 / 24000 / (line["ms_per_step"] / 1e3)) / line["value"] < 1e-3


def test_bench_tp_groups_are_replicas():
    """--gpus 4 --tp 2: two TP groups of consecutive ranks = 2 replicas."""
    rc, line, err = _run_bench(["--gpus", "4", "--tp", "2", "--plumbing", "--steps", "5"])
    assert rc == 0, err[-2000:]
    assert line["n_gpus"] == 4 and line["config"]["parallelism"] == "dp2, tp2"
    # the collective-share field --tp adds (plumbing pass: 1 ms, 0.75 ms without the "collective")
    tc = line["tp_collective"]
    assert tc["allreduce_calls_per_pass"] == 4
    assert 900 <= tc["lm_pass_us"] and 650 <= tc["lm_pass_us_null_collective"] < tc["lm_pass_us"]
    assert abs(tc["allreduce_us_per_pass"] - (tc["lm_pass_us"] - tc["lm_pass_us_null_collective"])) < 0.02
    assert 0 < tc["allreduce_share"] < 1


def test_bench_world_size_mismatch_refused():
    rc, line, err = _run_bench(["--gpus", "2", "--plumbing"], env_extra=dict(WORLD_SIZE="1", RANK="0",
                                                                                LOCAL_RANK="0"))
    assert rc != 0 and line is None and "WORLD_SIZE=1" in err


class _FakeEngine:
    """Stands in for vibevoice_amd.engine.Engine (no GPU): records how the
    model wires its TP rank into the engine."""
    made = []

    def __init__(self, cfg, sd, device, max_batch, max_ctx, tp_rank=0, tp_size=1, tp_unique_id=None, tp_head=False,
                 persistent=True):
        self.args = dict(tp_rank=tp_rank, tp_size=tp_size, uid=tp_unique_id, tp_head=tp_head)
        self.schedule = None
        self.max_batch = max_batch

    @staticmethod
    def tp_unique_id():
        return f"uid-of-global-rank-{torch.distributed.get_rank()}".encode()


def _tp_worker(rank, world, T, port, out):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    w, r, _, _ = bench.dist_setup()
    from tiny import tiny_config
    from vibevoice_amd import modeling_vibevoice_inference as mvi
    mvi.Engine = _FakeEngine
    group, replica, replicas = bench.tp_groups(w, r, T)
    m = mvi.VibeVoiceForConditionalGenerationInference(tiny_config(), {}, "cpu", tp_group=group)
    out[rank] = (replica, replicas, m.tp_rank, m.tp_size, m.engine.args["tp_rank"], m.engine.args["tp_size"],
                 m.engine.args["uid"], m.engine.args["tp_head"])
    torch.distributed.destroy_process_group()


def test_model_tp_wiring_world4_tp2():
    """The model-level TP wiring bench.py uses (gloo, 4 ranks, --tp 2): groups
    {0,1} and {2,3}, group-local ranks into the engine, and the RCCL unique id
    made by each group's first rank broadcast to its peers only
    (modeling_vibevoice_inference.py __init__)."""
    port = _free_port()
    with mp.Manager() as m:
        out = m.dict()
        mp.spawn(_tp_worker, args=(4, 2, port, out), nprocs=4, join=True)
        res = dict(out)
    for r in range(4):
        replica, replicas, tr, ts, etr, ets, uid, th = res[r]
        assert th is False      # tiny_config's head is cache-resident: replicated (head_tp_default)
        assert (replica, replicas) == (r // 2, 2)
        assert tr == etr == r % 2 and ts == ets == 2
        assert uid == f"uid-of-global-rank-{2 * (r // 2)}".encode()
