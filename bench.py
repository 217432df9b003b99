#!/usr/bin/env python3
"""Benchmark: GRI-Mech 3.0 constant-pressure ignition sweep on MI355X (BASELINE.json metric).

One "step" = one ckmi_reactor_run over this rank's shard of the ignition-delay sweep
(configs[2]: 64 T0 x 32 phi x 32 P = 65,536 CONP adiabatic CH4/air reactors per GPU,
t_end = 1 s, TIFP ignition, ATOL/RTOL = 1e-10/1e-8).  For N GPUs the sweep has 64*N
temperatures and rank r takes every N-th one (weak scaling, no collectives on the data path).
Inputs are resident in HBM before the timed region.  value = reactors integrated by all
ranks / max-over-ranks wall time.

Also reported: the ROP+thermo evaluation rate (configs[1], random (T, P, Y) states), a
roofline object for the reactor kernel (algorithmic FLOPs from solver statistics, see
pychemkin_amd/perf.py) and the CPU baseline (oracle/ C restatement, OpenMP, timed on a
strided sample of the same sweep on this host).

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from pychemkin_amd import _native  # noqa: E402
from pychemkin_amd.mechanism import Mechanism  # noqa: E402
from pychemkin_amd.perf import count_ops, reactor_flops  # noqa: E402

P_ATM = 1.01325e6
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) peak, MI355X_MICROARCH.md / SURVEY 8d
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak
# HBM traffic per launch from rocprofv3 PMC passes of this same bench workload (FETCH_SIZE x2 per the
# gfx950 calibration + WRITE_SIZE; scripts/pmc_traffic.sh -> scripts/traffic_summary.py)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")


def load_traffic(kernel: str, units: int):
    """Measured HBM bytes per launch of `kernel` for a launch of `units` units, or None."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)[kernel]
    except (OSError, KeyError, ValueError):
        return None
    if int(t.get("units", -1)) != int(units):
        return None
    return float(t["bytes_per_launch"])


def mechanism():
    return Mechanism.from_files(os.path.join(ROOT, "data", "grimech30_chem.inp"),
                                os.path.join(ROOT, "data", "grimech30_thermo.dat"))


def ch4_air_Y(mech, phi):
    """CH4/air at equivalence ratio phi (X_by_Equivalence_Ratio, mixture.py:2383-2539), mass fractions."""
    KK = mech.KK
    iCH4, iO2, iN2 = mech.species.index("CH4"), mech.species.index("O2"), mech.species.index("N2")
    alpha = 2.0 / 0.21
    X = np.zeros((len(phi), KK))
    X[:, iCH4] = phi
    X[:, iO2] = 0.21 * alpha
    X[:, iN2] = 0.79 * alpha
    X /= X.sum(axis=1, keepdims=True)
    Y = X * mech.wt
    return Y / Y.sum(axis=1, keepdims=True)


def sweep_c4(mech, world, rank):
    """configs[3]: 128 T0 x 64 phi x 64 P x {CONP, CONV} = 2^20 reactors in total, strided over ranks
    (strong scaling: the total is fixed).  problem = CONP for even, CONV for odd global index."""
    T = 1100.0 + 600.0 * np.arange(128) / 127
    phi = 0.5 + 1.5 * np.arange(64) / 63
    P = P_ATM * 10.0 ** (2.0 * np.arange(64) / 63)
    TT, FF, PP = np.meshgrid(T, phi, P, indexing="ij")
    TT, FF, PP = np.repeat(TT.ravel(), 2), np.repeat(FF.ravel(), 2), np.repeat(PP.ravel(), 2)
    prob = np.tile(np.array([1, 2], np.int32), TT.size // 2)
    sel = slice(rank, None, world)
    return TT[sel], PP[sel], ch4_air_Y(mech, FF[sel]), prob[sel]


def sweep(mech, world, rank, nT=64, nphi=32, nP=32):
    """Rank's shard of the (64*world) x 32 x 32 ignition sweep (configs[2] at world = 1)."""
    T_all = 1100.0 + 600.0 * np.arange(nT * world) / (nT * world - 1)
    T_sel = T_all[rank::world]
    phi = 0.5 + 1.5 * np.arange(nphi) / (nphi - 1)
    P = P_ATM * 10.0 ** (2.0 * np.arange(nP) / (nP - 1))
    TT, FF, PP = np.meshgrid(T_sel, phi, P, indexing="ij")
    TT, FF, PP = TT.ravel(), FF.ravel(), PP.ravel()
    return TT, PP, ch4_air_Y(mech, FF)


def rop_bench(dev, mech, ns, reps=3):
    """ROP + thermo over ns random (T, P, Y) states of `mech` (ckmi_rop_thermo), HIP-event timed."""
    tables = mech.to_tables()
    ops = count_ops(tables)
    dm = _native.DeviceMechanism(tables, device=dev)
    rng = np.random.default_rng(0)
    Ts = torch.as_tensor(rng.uniform(300.0, 3000.0, ns), device=dev)
    Ps = torch.as_tensor(P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, ns), device=dev)
    Ys = torch.as_tensor(rng.dirichlet(0.5 * np.ones(mech.KK), ns).T.copy(), device=dev)
    dm.rop_thermo(Ts, Ps, Ys)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dm.rop_thermo(Ts, Ps, Ys)
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / 1e3 / reps
    tf = ops["F_rop"] * ns / sec / 1e12
    return {"mechanism": f"synthetic GRI-3.0 + tracers, KK = {mech.KK}, II = {mech.II}", "states": ns,
            "value": ns / sec, "unit": "states/s", "ms_per_launch": sec * 1e3,
            "roofline": {"bound": "mfma", "pipe": "fp64-valu", "achieved": tf, "peak": FP64_PEAK_TFLOPS,
                         "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                         "hbm_GBs": ops["bytes_rop"] * ns / sec / 1e9, "traffic": load_traffic("rop_161sp", ns)}}


def lu_bench(dev, nsys, n):
    """Batched LU (ckmi_lu_factor_batched) on nsys Newton-like matrices I - gamma J of size n, timed with HIP
    events on the stream it is launched on; algorithmic work (2/3) n^3 per matrix."""
    g = torch.Generator(device=dev).manual_seed(0)
    A0 = torch.eye(n, dtype=torch.float64, device=dev) - 1e-6 * torch.randn(
        (nsys, n, n), dtype=torch.float64, device=dev, generator=g) * 10.0 ** (6.0 * torch.rand(
            (nsys, n, n), dtype=torch.float64, device=dev, generator=g))
    A = torch.empty_like(A0)
    times = []
    for it in range(4):
        A.copy_(A0)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        _, _, info = _native.lu_factor_batched(A)
        e1.record()
        torch.cuda.synchronize()
        if it:
            times.append(e0.elapsed_time(e1) / 1e3)
    sec = float(np.median(times))
    flops = nsys * 2.0 / 3.0 * n ** 3
    nbytes = nsys * 2.0 * n * n * 8
    del A, A0
    return {"kernel": "lu_factor_kernel<11>", "systems": nsys, "n": n, "ms_per_launch": sec * 1e3,
            "systems_per_s": nsys / sec, "singular": int((info != 0).sum().item()),
            "roofline": {"bound": "mfma", "pipe": "fp64-mfma", "achieved": flops / sec / 1e12,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": flops / sec / 1e12 / FP64_PEAK_TFLOPS,
                         "hbm_GBs": nbytes / sec / 1e9, "traffic": load_traffic("lu", nsys)}}


RUN = dict(energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reactors", type=int, default=0, help="override reactors per GPU (0 = full 65,536 shard)")
    ap.add_argument("--rop-states", type=int, default=10_000_000)
    ap.add_argument("--lu-systems", type=int, default=16384,
                    help="configs[4] component: batched n = 161 Newton-matrix LU on MFMA (0 = skip)")
    ap.add_argument("--big-states", type=int, default=1_000_000,
                    help="configs[4] component: ROP+thermo on the synthetic 161-species mechanism (0 = skip)")
    ap.add_argument("--cpu-sample", type=int, default=16384, help="max reactors in the CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline time budget")
    ap.add_argument("--cpu-threads", type=int, default=0)
    ap.add_argument("--workload", choices=("c3", "c4"), default="c3",
                    help="c3: configs[2], 65,536 CONP reactors per GPU (weak scaling, the metric); "
                         "c4: configs[3], 2^20 CONP+CONV reactors in total (strong scaling)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    mech = mechanism()
    tables = mech.to_tables()
    ops = count_ops(tables)
    dm = _native.DeviceMechanism(tables, device=dev)

    if args.workload == "c4":
        T0, P0, Y0, prob = sweep_c4(mech, world, rank)
    else:
        T0, P0, Y0 = sweep(mech, world, rank)
        prob = np.ones(len(T0), np.int32)
    if args.reactors:
        T0, P0, Y0, prob = T0[: args.reactors], P0[: args.reactors], Y0[: args.reactors], prob[: args.reactors]
    n = len(T0)
    T0_d = torch.as_tensor(T0, device=dev)
    P0_d = torch.as_tensor(P0, device=dev)
    V0_d = torch.ones(n, dtype=torch.float64, device=dev)
    Y0_d = torch.as_tensor(Y0, device=dev).contiguous()
    prob_d = torch.as_tensor(prob, device=dev)
    cfg = _native.make_cfg(**RUN)
    out = dict(tau=torch.empty(n, dtype=torch.float64, device=dev), T=torch.empty(n, dtype=torch.float64, device=dev),
               P=torch.empty(n, dtype=torch.float64, device=dev), V=torch.empty(n, dtype=torch.float64, device=dev),
               Y=torch.empty((n, mech.KK), dtype=torch.float64, device=dev),
               stats=torch.empty((n, _native.NSTAT), dtype=torch.int32, device=dev))

    def step():
        return dm.reactor_run(cfg, prob_d, T0_d, P0_d, V0_d, Y0_d, out=out)

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]
    t0 = time.perf_counter()
    for k in range(args.steps):
        ev[k][0].record()
        res = step()
        ev[k][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    tmax = tmax.item()

    stats = res["stats"].cpu().numpy()
    tau = res["tau"].cpu().numpy()
    nbad = int((stats[:, 6] != 0).sum())
    nnoign = int((tau <= 0).sum())
    flops = reactor_flops(ops, stats)
    kern_s = float(np.mean(kern_ms)) / 1e3
    achieved_tf = flops / kern_s / 1e12

    total_reactors = n * world * args.steps
    value = total_reactors / tmax

    # PCIe-inclusive rate (reported beside value, never as value): host numpy inputs -> H2D ->
    # one launch -> D2H of tau, T, P, V, Y, stats, on this rank
    torch.cuda.synchronize()
    tp = time.perf_counter()
    rp = dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0)
    host_out = {k: v.cpu().numpy() for k, v in rp.items()}
    torch.cuda.synchronize()
    pcie_s = time.perf_counter() - tp
    pcie = {"reactors_per_s": n / pcie_s, "seconds": pcie_s,
            "bytes_h2d": int(T0.nbytes + P0.nbytes + Y0.nbytes + prob.nbytes + 8 * n),
            "bytes_d2h": int(sum(a.nbytes for a in host_out.values()))}
    del rp, host_out

    # ---- ROP + thermo (configs[1]) : secondary metric
    rop = None
    if args.rop_states > 0:
        rng = np.random.default_rng(0)
        ns = args.rop_states
        Ts = torch.as_tensor(rng.uniform(300.0, 3000.0, ns), device=dev)
        Ps = torch.as_tensor(P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, ns), device=dev)
        Ys = torch.as_tensor(rng.dirichlet(0.5 * np.ones(mech.KK), ns).T.copy(), device=dev)
        wdot = torch.empty((mech.KK, ns), dtype=torch.float64, device=dev)
        cp = torch.empty(ns, dtype=torch.float64, device=dev)
        hh = torch.empty(ns, dtype=torch.float64, device=dev)
        dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh)
        torch.cuda.synchronize()
        reps = 3
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh)
        e1.record()
        torch.cuda.synchronize()
        sec = e0.elapsed_time(e1) / 1e3 / reps
        rop = {
            "value": ns / sec, "unit": "states/s", "states": ns, "ms_per_launch": sec * 1e3,
            "roofline": {
                "bound": "mfma", "pipe": "fp64-valu", "achieved": ops["F_rop"] * ns / sec / 1e12,
                "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                "frac": ops["F_rop"] * ns / sec / 1e12 / FP64_PEAK_TFLOPS,
                "hbm_GBs": ops["bytes_rop"] * ns / sec / 1e9, "hbm_frac": ops["bytes_rop"] * ns / sec / 1e9 / HBM_PEAK_GBS,
                "traffic": load_traffic("rop", ns),
            },
            "cpu_baseline": None,
        }
        if rank == 0 and world == 1 and args.cpu_sample > 0:
            # oracle C restatement over the first 200k of the same states (OpenMP over states), and
            # over the first 20k on one core; the GPU result of the same states is the checker
            from oracle.oracle import Oracle  # noqa: E402  (cpu_baseline leg only)
            orc_r = Oracle(mech)
            threads = args.cpu_threads or min(16, os.cpu_count() or 1)
            m = min(ns, 200_000)
            Th, Ph, Yh = Ts[:m].cpu().numpy(), Ps[:m].cpu().numpy(), Ys[:, :m].cpu().numpy()
            tc = time.perf_counter()
            wc, _, _ = orc_r.rop_batch(Th, Ph, Yh, nthreads=threads)
            t_all = time.perf_counter() - tc
            m1 = min(m, 20_000)
            tc = time.perf_counter()
            orc_r.rop_batch(Th[:m1], Ph[:m1], np.ascontiguousarray(Yh[:, :m1]), nthreads=1)
            t_one = time.perf_counter() - tc
            wg = wdot[:, :m].cpu().numpy()
            rop["cpu_baseline"] = {
                "value": m / t_all, "unit": "states/s", "cores": threads, "kind": "port",
                "single_core_value": m1 / t_one,
                "sample": f"first {m} of the same 10M states ({m1} on one core), oracle C restatement, OpenMP over states",
                "wdot_max_rel_diff_vs_gpu": float(np.max(np.abs(wg - wc) / np.max(np.abs(wc), axis=0, keepdims=True))),
            }
        del Ts, Ps, Ys, wdot, cp, hh

    # ---- configs[4] component: batched FP64 LU of n = 161 Newton matrices (MFMA trailing updates)
    lu = None
    if rank == 0 and args.lu_systems > 0:
        lu = lu_bench(dev, args.lu_systems, 161)

    rop_big = None
    if rank == 0 and args.big_states > 0:
        rop_big = rop_bench(dev, Mechanism.from_files(os.path.join(ROOT, "data", "gri30_tracer161_chem.inp"),
                                                      os.path.join(ROOT, "data", "gri30_tracer161_thermo.dat")),
                            args.big_states)

    # ---- CPU baseline (rank 0, N = 1): oracle C restatement on a strided sample
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        from oracle.oracle import Oracle  # noqa: E402  (cpu_baseline leg only)
        orc = Oracle(mech)
        # strided sample of the same sweep, processed in chunks until ~cpu_seconds of CPU work
        stride = max(1, n // args.cpu_sample)
        order = np.random.default_rng(0).permutation(np.arange(0, n, stride)[: args.cpu_sample])
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        chunk = 32 * threads
        done, tcpu, dmax = 0, 0.0, 0.0
        while done < order.size and tcpu < args.cpu_seconds:
            idx = order[done: done + chunk]
            tc = time.perf_counter()
            nfail, cres, _ = orc.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx],
                                               V0=np.ones(len(idx)), nthreads=threads, **RUN)
            tcpu += time.perf_counter() - tc
            ctau = np.array([r.tau for r in cres])
            dmax = max(dmax, float(np.max(np.abs(tau[idx] / ctau - 1))))
            done += len(idx)
        # the same oracle on one core, over the first chunk of the sample (~3 s)
        idx1 = order[: max(8, min(64, order.size))]
        tc = time.perf_counter()
        orc.reactor_batch(T0[idx1], P0[idx1], Y0[idx1], problem=prob[idx1], V0=np.ones(len(idx1)), nthreads=1, **RUN)
        one_core = len(idx1) / (time.perf_counter() - tc)
        cpu = {"value": done / tcpu, "unit": "reactors/s", "cores": threads, "kind": "port",
               "single_core_value": one_core, "single_core_sample": f"{len(idx1)} reactors of the same sample",
               "sample": f"{done} reactors (random subset of every {stride}th of this GPU's sweep), oracle C restatement, "
                         f"OpenMP over reactors",
               "tau_max_rel_diff_vs_gpu": dmax,
               "seconds": tcpu}

    if rank == 0:
        line = {
            "metric": "reactor integrations/sec (GRI-3.0 const-P ignition)",
            "value": value,
            "unit": "reactors/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": tmax / args.steps * 1e3,
            "higher_is_better": True,
            "scaling": "weak" if args.workload == "c3" else "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": ("configs[2]: GRI-3.0 CONP CH4/air ignition sweep 64 T0 x 32 phi x 32 P per GPU"
                                    if args.workload == "c3" else
                                    "configs[3]: GRI-3.0 CH4/air 128 T0 x 64 phi x 64 P x {CONP, CONV} = 2^20 "
                                    "reactors in total"),
                       "reactors_per_gpu": n, "t_end_s": 1.0, "atol": 1e-10, "rtol": 1e-8, "ignition": "TIFP",
                       "parallelism": f"shard-by-condition x{world}"},
            "reactors_per_min": value * 60.0,
            "failed_reactors": nbad,
            "not_ignited": nnoign,
            "solver": {"mean_steps": float(stats[:, 0].mean()), "mean_rhs": float(stats[:, 1].mean()),
                       "mean_jac": float(stats[:, 2].mean()), "mean_lu": float(stats[:, 3].mean()),
                       "mean_newton": float(stats[:, 7].mean())},
            "roofline": {"bound": "mfma", "pipe": "fp64-valu", "kernel": "reactor_kernel<54>",
                         "achieved": achieved_tf, "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved_tf / FP64_PEAK_TFLOPS, "traffic": load_traffic("reactor", n),
                         "flops_per_launch": flops, "kernel_ms": kern_s * 1e3},
            "cpu_baseline": cpu,
            "rop": rop,
            "lu": lu,
            "rop_161sp": rop_big,
            "pcie_inclusive": pcie,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
