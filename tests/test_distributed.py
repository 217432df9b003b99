"""Multi-rank sharding of the sweep (world_size 2, gloo, CPU): the N>1 bench / BatchSweep path.

The path shards by condition with no data-path collective; the only collectives are the
timing barrier and the max-over-ranks reduction.  Ranks run the CPU oracle here in place of
the GPU (this test checks the partitioning and the reduction, not the kernels).
"""
import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch

    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    from oracle.oracle import Oracle

    mech = bench.mechanism()
    T0, P0, Y0, _ = bench.sweep(mech, world, rank, nT=4, nphi=2, nP=2)
    orc = Oracle(mech)
    _, res, Yend = orc.reactor_batch(T0, P0, Y0, problem=np.ones(len(T0), np.int32), V0=np.ones(len(T0)),
                                     nthreads=1, energy=1, t_end=0.05, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    tau = np.array([r.tau for r in res])
    t = torch.tensor([float(rank + 1)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    dist.barrier()
    q.put((rank, T0.tolist(), P0.tolist(), Y0[:, 3].tolist(), tau.tolist(), float(t.item())))
    dist.destroy_process_group()


def test_two_rank_shards_partition_the_sweep_and_match_single_rank():
    import bench

    world = 2
    port = _free_port()
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    outs = [q.get(timeout=300) for _ in range(world)]
    for p in ps:
        p.join(timeout=60)
        assert p.exitcode == 0
    outs.sort()
    assert all(o[5] == 2.0 for o in outs)  # max-over-ranks reduction
    mech = bench.mechanism()
    T_f, P_f, Y_f, _ = bench.sweep(mech, 1, 0, nT=8, nphi=2, nP=2)
    key = lambda T, P, yo2: (T, P, yo2)  # (T0, P0, Y_O2) identifies a condition (phi sets Y_O2)
    got = sorted(key(*c) for o in outs for c in zip(o[1], o[2], o[3]))
    assert got == sorted(key(*c) for c in zip(T_f.tolist(), P_f.tolist(), Y_f[:, 3].tolist()))  # disjoint, complete
    # shard invariance: the same condition gives the same tau on either rank layout
    from oracle.oracle import Oracle

    orc = Oracle(mech)
    T0, P0, Y0, _ = bench.sweep(mech, 1, 0, nT=8, nphi=2, nP=2)
    _, res, _ = orc.reactor_batch(T0, P0, Y0, problem=np.ones(len(T0), np.int32), V0=np.ones(len(T0)), nthreads=1,
                                  energy=1, t_end=0.05, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    full = {key(a, b, c): r.tau for a, b, c, r in zip(T0.tolist(), P0.tolist(), Y0[:, 3].tolist(), res)}
    for o in outs:
        for a, b, c, t in zip(o[1], o[2], o[3], o[4]):
            assert full[key(a, b, c)] == t


@pytest.mark.parametrize("world", [2, 4, 8])
def test_secondary_sweeps_partition_over_ranks(world):
    """configs[3] (2^20 GRI reactors) and configs[4] (262,144 stand-in reactors) are strong-scaling
    sweeps: the ranks' strided shards are disjoint and together are exactly the single-rank sweep."""
    import bench

    mech = bench.mechanism()
    T1, P1, Y1, pr1 = bench.sweep_c4(mech, 1, 0)
    assert T1.size == 2 ** 20 and set(np.unique(pr1)) == {1, 2}
    parts = [bench.sweep_c4(mech, world, r) for r in range(world)]
    assert sum(p[0].size for p in parts) == T1.size
    for r, p in enumerate(parts):
        assert np.array_equal(p[0], T1[r::world]) and np.array_equal(p[3], pr1[r::world])
        assert np.array_equal(p[2], Y1[r::world])
    big = bench.big_mechanism()
    T5, P5, Y5, _ = bench.sweep_c5(big, 1, 0)
    assert T5.size == 262144 and np.all(Y5[:, big.species.index("AX1")] > 0)
    parts = [bench.sweep_c5(big, world, r) for r in range(world)]
    assert sum(p[0].size for p in parts) == T5.size
    for r, p in enumerate(parts):
        assert np.array_equal(p[1], P5[r::world])


@pytest.mark.parametrize("n", [2, 4])
def test_bench_launcher_shards_and_max_time(n):
    """bench.py --gpus N run directly is its own launcher (no external torchrun): it starts N rank
    processes, the headline shards are disjoint and together complete (64 N x 32 x 32 reactors, the
    strided T0 split), and the reported time is the max over ranks.  --plan runs the same launcher
    and timing protocol on CPU (gloo)."""
    import json
    import subprocess
    import sys

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(n), "--plan"], env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr[-2000:]
    rep = json.loads(out.stdout.strip().splitlines()[-1])
    assert rep["n_ranks"] == n and rep["shard_sizes"] == [65536] * n
    assert rep["disjoint"] and rep["complete"]
    assert rep["max_seconds"] >= max(rep["rank_seconds"]) - 1e-9
    assert rep["max_seconds"] >= 0.05 * n


def test_bench_launcher_refuses_more_gpus_than_visible():
    import subprocess
    import sys

    import torch

    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    n = torch.cuda.device_count() + 1
    out = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", str(max(n, 2)), "--steps", "1"],
                         env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0 and "visible" in (out.stderr + out.stdout)
