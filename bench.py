#!/usr/bin/env python3
"""Benchmark: GRI-Mech 3.0 constant-pressure ignition sweep on MI355X (BASELINE.json metric).

Headline (`value`): configs[2] -- one "step" = one ckmi_reactor_run over this rank's shard of the
ignition-delay sweep, 64 T0 x 32 phi x 32 P = 65,536 CONP adiabatic CH4/air reactors per GPU,
t_end = 1 s, TIFP ignition, ATOL/RTOL = 1e-10/1e-8.  For N GPUs the sweep has 64*N temperatures
and rank r takes every N-th one (weak scaling, no collectives on the data path).  Inputs are
resident in HBM before the timed region; value = reactors integrated by all ranks / max-over-ranks
wall time.  PCIe transfers are excluded from `value`; the PCIe-inclusive rate of the same launch is
reported beside it (`pcie_inclusive`).

Secondary lines in the same JSON object (each sharded over the ranks, max-over-ranks timing):
  c1   configs[0]: ONE GRI-3.0 CONP reactor (CH4/air phi 1, 1200 K, 1 atm, TIFP, 1e-10/1e-8) through the
       drop-in GivenPressureBatchReactor_EnergyConservation.run(): per-call wall latency (median of 7),
       solver counts, the oracle on one core; plus the reference's serial 20-condition loop
       (ignitiondelay.py:127-144) against one BatchSweep launch of the same 20 (rank 0 only)
  c4   configs[3]: 2^20 GRI-3.0 reactors, CONP/CONV alternating, strong scaling (total fixed)
  c5   configs[4]: 262,144 reactors of the 161-species stand-in mechanism (no ~160-species
       n-heptane mechanism exists offline; parity with Chemkin unpinned), workgroup-per-reactor
       kernel, strong scaling
  rop  configs[1]: ROP + thermo of 10M random (T, P, Y) states
  lu / rop_161sp: configs[4] components (batched MFMA LU, 161-species ROP)
  rop_ext161  the specialised ROP kernel on the extended 161-species stand-in (PLOG, HIGH, FORD /
       RORD, fractional and wide reactions: every reaction form since round 3)
  pfr  4,096 GRI-3.0 plug-flow tubes (problem 3, 1 cm at 1 cm/s), FP64-inverse wave kernel
  hcci 15,625 single-zone HCCI cylinders (problem 4, the hcciengine golden's engine with its
       ICHX / Woschni wall heat transfer, -142 .. 116 CA), FP64-inverse wave kernel
Each carries a roofline object (algorithmic FLOPs from the solver statistics, pychemkin_amd/perf.py,
over the kernel time measured with HIP events on the launch stream) and, on rank 0 at N = 1, a
CPU baseline: the oracle C restatement (OpenMP) timed on a bounded sample of the same workload on
this host.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W] [--lines c1,c3,c4,c5,rop,lu,rop161,ropext,pfr,hcci]

Launch: under torch.distributed.run (RANK / WORLD_SIZE / LOCAL_RANK set) every process is one
rank.  Run directly with --gpus N > 1, bench.py is its own launcher: it starts N child processes
(one GPU each, same arguments, MASTER_ADDR 127.0.0.1) before anything touches a GPU, forwards
rank 0's JSON line and exits with the worst child status; N above the visible devices is an error.
--plan prints the shard layout and the max-over-ranks timing path without a GPU (gloo).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
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
FP64_PEAK_TFLOPS = 78.6   # MI355X FP64 vector (= FP64 matrix) peak, SURVEY 8d
HBM_PEAK_GBS = 8000.0     # MI355X HBM3E peak
# HBM traffic per launch from rocprofv3 PMC passes of this same bench workload (FETCH_SIZE x2 per the
# gfx950 calibration + WRITE_SIZE; scripts/pmc_traffic.sh -> scripts/traffic_summary.py)
TRAFFIC_FILE = os.path.join(ROOT, "profiles", "traffic.json")
RUN = dict(energy=1, t_end=1.0, atol=1e-10, rtol=1e-8, ign_mode="TIFP")


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


def cpu_threads():
    """Threads for the CPU baseline: the OpenMP allotment of this job (the GPU box sets
    OMP_NUM_THREADS to its CPU share), else every CPU of the host; nproc is reported beside it."""
    env = os.environ.get("OMP_NUM_THREADS")
    return int(env) if env and env.isdigit() and int(env) > 0 else (os.cpu_count() or 1)


def host_info():
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"nproc": os.cpu_count(), "affinity_cpus": aff, "omp_num_threads": os.environ.get("OMP_NUM_THREADS")}


def mechanism():
    return Mechanism.from_files(os.path.join(ROOT, "data", "grimech30_chem.inp"),
                                os.path.join(ROOT, "data", "grimech30_thermo.dat"))


def big_mechanism():
    return Mechanism.from_files(os.path.join(ROOT, "data", "gri30_tracer161_chem.inp"),
                                os.path.join(ROOT, "data", "gri30_tracer161_thermo.dat"))


def ch4_air_Y(mech, phi, tracer=0.0):
    """CH4/air at equivalence ratio phi (X_by_Equivalence_Ratio, mixture.py:2383-2539), mass
    fractions; tracer > 0 replaces that fraction of the N2 by AX1 (161-species stand-in)."""
    KK = mech.KK
    iCH4, iO2, iN2 = mech.species.index("CH4"), mech.species.index("O2"), mech.species.index("N2")
    X = np.zeros((len(phi), KK))
    X[:, iCH4] = phi
    X[:, iO2] = 2.0
    X[:, iN2] = 2.0 * 0.79 / 0.21 * (1.0 - tracer)
    if tracer > 0.0:
        X[:, mech.species.index("AX1")] = 2.0 * 0.79 / 0.21 * tracer
    X /= X.sum(axis=1, keepdims=True)
    Y = X * mech.wt
    return Y / Y.sum(axis=1, keepdims=True)


def sweep_index(world, rank, nT=64, nphi=32, nP=32):
    """Global reactor indices (iT, iphi, iP flattened over the 64*world x 32 x 32 sweep) of rank's
    shard, in the order sweep() lays them out."""
    iT = np.arange(nT * world)[rank::world]
    I, F, Q = np.meshgrid(iT, np.arange(nphi), np.arange(nP), indexing="ij")
    return (I.ravel() * nphi + F.ravel()) * nP + Q.ravel()


def sweep(mech, world, rank, nT=64, nphi=32, nP=32):
    """Rank's shard of the (64*world) x 32 x 32 ignition sweep (configs[2] at world = 1)."""
    T_all = 1100.0 + 600.0 * np.arange(nT * world) / (nT * world - 1)
    T_sel = T_all[rank::world]
    phi = 0.5 + 1.5 * np.arange(nphi) / (nphi - 1)
    P = P_ATM * 10.0 ** (2.0 * np.arange(nP) / (nP - 1))
    TT, FF, PP = np.meshgrid(T_sel, phi, P, indexing="ij")
    TT, FF, PP = TT.ravel(), FF.ravel(), PP.ravel()
    return TT, PP, ch4_air_Y(mech, FF), np.ones(TT.size, np.int32)


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


def sweep_c5(mech, world, rank):
    """configs[4] on the 161-species stand-in: 64 T0 x 64 phi x 64 P = 262,144 CONP reactors in total
    (strong scaling), T0 1100-1700 K (the stand-in's chemistry is CH4's: the n-heptane grid's
    700-1300 K would not ignite), phi 0.5-2, P 10-60 atm, 20 % of the N2 replaced by the tracer AX1
    so the tracer exchange chemistry is live.  Strided over ranks."""
    T = 1100.0 + 600.0 * np.arange(64) / 63
    phi = 0.5 + 1.5 * np.arange(64) / 63
    P = P_ATM * (10.0 + 50.0 * np.arange(64) / 63)
    TT, FF, PP = np.meshgrid(T, phi, P, indexing="ij")
    TT, FF, PP = TT.ravel(), FF.ravel(), PP.ravel()
    sel = slice(rank, None, world)
    return TT[sel], PP[sel], ch4_air_Y(mech, FF[sel], tracer=0.2), np.ones(TT[sel].size, np.int32)


class Shard:
    """One rank's reactors of a sweep, resident in HBM, with preallocated outputs."""

    def __init__(self, dm, dev, T0, P0, Y0, prob):
        self.dm, self.dev, self.n = dm, dev, len(T0)
        self.host = (T0, P0, Y0, prob)
        f64 = dict(dtype=torch.float64, device=dev)
        self.T0 = torch.as_tensor(T0, device=dev)
        self.P0 = torch.as_tensor(P0, device=dev)
        self.V0 = torch.ones(self.n, **f64)
        self.Y0 = torch.as_tensor(Y0, device=dev).contiguous()
        self.prob = torch.as_tensor(prob, device=dev)
        self.out = dict(tau=torch.empty(self.n, **f64), T=torch.empty(self.n, **f64), P=torch.empty(self.n, **f64),
                        V=torch.empty(self.n, **f64), Y=torch.empty((self.n, dm.KK), **f64),
                        stats=torch.empty((self.n, _native.NSTAT), dtype=torch.int32, device=dev),
                        t_stop=torch.empty(self.n, **f64))

    def step(self, cfg, lo=0, hi=None):
        if hi is None:
            return self.dm.reactor_run(cfg, self.prob, self.T0, self.P0, self.V0, self.Y0, out=self.out)
        return self.dm.reactor_run(cfg, self.prob[lo:hi], self.T0[lo:hi], self.P0[lo:hi], self.V0[lo:hi],
                                   self.Y0[lo:hi])


def timed(world, fn, steps):
    """Run fn() `steps` times between barrier + synchronize fences; returns (max-over-ranks wall
    seconds, per-launch HIP-event milliseconds on the launch stream, last result)."""
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    t0 = time.perf_counter()
    res = None
    for k in range(steps):
        ev[k][0].record()
        res = fn()
        ev[k][1].record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in ev]
    tmax = torch.tensor([elapsed], dtype=torch.float64, device=torch.cuda.current_device())
    if world > 1:
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
    return tmax.item(), kern_ms, res


def solver_summary(stats):
    return {"mean_steps": float(stats[:, 0].mean()), "mean_rhs": float(stats[:, 1].mean()),
            "mean_jac": float(stats[:, 2].mean()), "mean_lu": float(stats[:, 3].mean()),
            "mean_newton": float(stats[:, 7].mean())}


def reactor_roofline(ops, stats, kern_s, kernel, traffic_key, n):
    flops = reactor_flops(ops, stats)
    tf = flops / kern_s / 1e12
    return {"bound": "valu", "pipe": "fp64-valu", "kernel": kernel, "achieved": tf, "peak": FP64_PEAK_TFLOPS,
            "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS, "traffic": load_traffic(traffic_key, n),
            "flops_per_launch": flops, "flops_per_reactor": flops / n, "kernel_ms": kern_s * 1e3}


def cpu_reactor_baseline(mech, T0, P0, Y0, prob, tau_gpu, seconds, max_sample, single=True, run=None):
    """Oracle C restatement (OpenMP over reactors) on a random subset of a strided sample of the same
    sweep, in chunks until ~seconds of CPU work; plus the same oracle on one core.  run: the oracle's
    configuration when it is not the bench's RUN (plug-flow tubes, engine cylinders)."""
    from oracle.oracle import Oracle  # noqa: E402  (cpu_baseline leg only)

    run = RUN if run is None else run
    orc = Oracle(mech)
    n = len(T0)
    stride = max(1, n // max_sample)
    order = np.random.default_rng(0).permutation(np.arange(0, n, stride)[:max_sample])
    threads = cpu_threads()
    chunk = 32 * threads
    done, tcpu, dmax = 0, 0.0, 0.0
    while done < order.size and tcpu < seconds:
        idx = order[done: done + chunk]
        tc = time.perf_counter()
        _, cres, _ = orc.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(len(idx)),
                                       nthreads=threads, **run)
        tcpu += time.perf_counter() - tc
        ctau = np.array([r.tau for r in cres])
        ok = ctau > 0
        if ok.any():
            dmax = max(dmax, float(np.max(np.abs(tau_gpu[idx][ok] / ctau[ok] - 1))))
        done += len(idx)
    out = {"value": done / tcpu, "unit": "reactors/s", "cores": threads, "kind": "port", "host": host_info(),
           "sample": f"{done} reactors (random subset of every {stride}th reactor of this GPU's sweep), "
                     f"oracle C restatement, OpenMP over reactors",
           "tau_max_rel_diff_vs_gpu": dmax, "seconds": tcpu}
    if single:
        idx1 = order[: max(4, min(32, order.size))]
        tc = time.perf_counter()
        orc.reactor_batch(T0[idx1], P0[idx1], Y0[idx1], problem=prob[idx1], V0=np.ones(len(idx1)), nthreads=1, **run)
        out["single_core_value"] = len(idx1) / (time.perf_counter() - tc)
        out["single_core_sample"] = f"{len(idx1)} reactors of the same sample, 1 thread"
    return out


def rop_line(dev, mech, ops, ns, rank, world, cpu_sample, kernel_name="rop_kernel<0,1>", traffic_key="rop",
             label=None):
    """ROP + thermo over ns random (T, P, Y) states (ckmi_rop_thermo), HIP-event timed."""
    dm = _native.DeviceMechanism(mech.to_tables(), device=dev)
    rng = np.random.default_rng(0)
    Ts = torch.as_tensor(rng.uniform(300.0, 3000.0, ns), device=dev)
    Ps = torch.as_tensor(P_ATM * 10.0 ** rng.uniform(-1.0, 2.0, ns), device=dev)
    Ys = torch.as_tensor(rng.dirichlet(0.5 * np.ones(mech.KK), ns).T.copy(), device=dev)
    wdot = torch.empty((mech.KK, ns), dtype=torch.float64, device=dev)
    cp = torch.empty(ns, dtype=torch.float64, device=dev)
    hh = torch.empty(ns, dtype=torch.float64, device=dev)
    dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh)  # warm-up: also compiles the specialised kernel (hipRTC)
    torch.cuda.synchronize()
    jit = dm.rop_jit_state() == 1
    if jit:
        kernel_name, flops_key, traffic_key = f"ckjit_rop_k{mech.KK}_i{mech.II}", "F_rop_jit", traffic_key + "_jit"
    else:
        flops_key = "F_rop"
    reps = 3
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        dm.rop_thermo(Ts, Ps, Ys, wdot, cp, hh)
    e1.record()
    torch.cuda.synchronize()
    sec = e0.elapsed_time(e1) / 1e3 / reps
    tf = ops[flops_key] * ns / sec / 1e12
    gbs = ops["bytes_rop"] * ns / sec / 1e9
    out = {"value": ns / sec, "unit": "states/s", "states": ns, "ms_per_launch": sec * 1e3,
           "roofline": {"bound": "valu", "pipe": "fp64-valu", "kernel": kernel_name, "achieved": tf,
                        "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": tf / FP64_PEAK_TFLOPS,
                        "hbm_GBs": gbs, "hbm_frac": gbs / HBM_PEAK_GBS, "traffic": load_traffic(traffic_key, ns)},
           "cpu_baseline": None,
           "kernel": "mechanism-specialised, one state per lane (hipRTC)" if jit else "generic, one reaction per lane"}
    if label:
        out["mechanism"] = label
    if rank == 0 and world == 1 and cpu_sample > 0:
        from oracle.oracle import Oracle  # noqa: E402  (cpu_baseline leg only)

        orc_r = Oracle(mech)
        threads = cpu_threads()
        small = mech.KK <= 63  # bounded sample: ~0.1-5 s of CPU work per leg
        m = min(ns, 200_000 if small else 100_000)
        Th, Ph, Yh = Ts[:m].cpu().numpy(), Ps[:m].cpu().numpy(), Ys[:, :m].cpu().numpy()
        tc = time.perf_counter()
        wc, _, _ = orc_r.rop_batch(Th, Ph, Yh, nthreads=threads)
        t_all = time.perf_counter() - tc
        m1 = min(m, 20_000 if small else 4_000)
        tc = time.perf_counter()
        orc_r.rop_batch(Th[:m1], Ph[:m1], np.ascontiguousarray(Yh[:, :m1]), nthreads=1)
        t_one = time.perf_counter() - tc
        wg = wdot[:, :m].cpu().numpy()
        out["cpu_baseline"] = {
            "value": m / t_all, "unit": "states/s", "cores": threads, "kind": "port", "host": host_info(),
            "single_core_value": m1 / t_one,
            "sample": f"first {m} of the same {ns} states ({m1} on one core), oracle C restatement, OpenMP over states",
            "wdot_max_rel_diff_vs_gpu": float(np.max(np.abs(wg - wc) / np.max(np.abs(wc), axis=0, keepdims=True))),
        }
    del Ts, Ps, Ys, wdot, cp, hh
    dm.close()
    return out


def lu_line(dev, nsys, n, cpu_sample=0):
    """Batched LU (ckmi_lu_factor_batched) on nsys Newton-like matrices I - gamma J of size n, timed with HIP
    events on the stream it is launched on; algorithmic work (2/3) n^3 per matrix.  cpu_baseline: the
    oracle's dense LU (the C integrator's own factorisation) over the first matrices, OpenMP over systems."""
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
        _, ipiv, info = _native.lu_factor_batched(A)
        e1.record()
        torch.cuda.synchronize()
        if it:
            times.append(e0.elapsed_time(e1) / 1e3)
    sec = float(np.median(times))
    flops = nsys * 2.0 / 3.0 * n ** 3
    nbytes = nsys * 2.0 * n * n * 8
    cpu = None
    if cpu_sample > 0:
        from oracle.oracle import lu_factor_batch  # noqa: E402  (cpu_baseline leg only)

        m = min(nsys, 4096)
        Ah = A0[:m].cpu().numpy()
        threads = cpu_threads()
        tc = time.perf_counter()
        LUc, pc, _ = lu_factor_batch(Ah, threads)
        t_all = time.perf_counter() - tc
        m1 = min(m, 256)
        tc = time.perf_counter()
        lu_factor_batch(Ah[:m1], 1)
        t_one = time.perf_counter() - tc
        LUg, pg = A[:m].cpu().numpy(), ipiv[:m].cpu().numpy()
        cpu = {"value": m / t_all, "unit": "systems/s", "cores": threads, "kind": "port", "host": host_info(),
               "single_core_value": m1 / t_one,
               "sample": f"first {m} of the same {nsys} matrices ({m1} on one core), oracle C dense LU "
                         "(partial pivoting), OpenMP over systems",
               "pivots_identical_frac": float(np.mean(np.all(pc == pg, axis=1))),
               "factor_max_abs_diff_vs_gpu": float(np.max(np.abs(LUc - LUg)))}
    del A, A0
    return {"kernel": "lu_factor_kernel<11>", "systems": nsys, "n": n, "ms_per_launch": sec * 1e3,
            "systems_per_s": nsys / sec, "singular": int((info != 0).sum().item()),
            "roofline": {"bound": "mfma", "pipe": "fp64-mfma", "achieved": flops / sec / 1e12,
                         "peak": FP64_PEAK_TFLOPS, "unit": "TFLOP/s", "frac": flops / sec / 1e12 / FP64_PEAK_TFLOPS,
                         "hbm_GBs": nbytes / sec / 1e9, "traffic": load_traffic("lu", nsys)},
            "cpu_baseline": cpu}


def secondary_sweep(name, dm, dev, mech, ops, sweep_fn, world, rank, args, kernel, traffic_key, workload, scaling):
    """One timed launch over this rank's shard of a secondary sweep (c4 / c5), after a small warm-up."""
    T0, P0, Y0, prob = sweep_fn(mech, world, rank)
    if args.sub_reactors:
        T0, P0, Y0, prob = T0[: args.sub_reactors], P0[: args.sub_reactors], Y0[: args.sub_reactors], prob[
            : args.sub_reactors]
    sh = Shard(dm, dev, T0, P0, Y0, prob)
    cfg = _native.make_cfg(**RUN)
    sh.step(cfg, 0, min(sh.n, 256))  # warm-up launch (code objects, LDS configuration)
    tmax, kern_ms, res = timed(world, lambda: sh.step(cfg), 1)
    stats = res["stats"].cpu().numpy()
    tau = res["tau"].cpu().numpy()
    total = torch.tensor([sh.n], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(total)
    total = int(total.item())
    line = {"metric": f"reactor integrations/sec ({workload})", "value": total / tmax, "unit": "reactors/s",
            "reactors_total": total, "reactors_per_gpu": sh.n, "seconds": tmax, "scaling": scaling,
            "failed_reactors": int((stats[:, 6] != 0).sum()), "not_ignited": int((tau <= 0).sum()),
            "solver": solver_summary(stats),
            "roofline": reactor_roofline(ops, stats, float(np.mean(kern_ms)) / 1e3, kernel, traffic_key, sh.n),
            "cpu_baseline": None}
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        line["cpu_baseline"] = cpu_reactor_baseline(mech, T0, P0, Y0, prob, tau, args.cpu_seconds_secondary,
                                                    args.cpu_sample, single=True)
    del sh, res
    return line


def model_sweep(mech, world, rank, total, T_lo, T_hi, P_lo, P_hi, phi_lo, phi_hi):
    """A fixed-total (strong-scaling) T0 x phi x P grid of `total` reactors, strided over the ranks."""
    m = int(round(total ** (1.0 / 3.0)))
    T = T_lo + (T_hi - T_lo) * np.arange(m) / (m - 1)
    phi = phi_lo + (phi_hi - phi_lo) * np.arange(m) / (m - 1)
    P = P_lo + (P_hi - P_lo) * np.arange(m) / (m - 1)
    TT, FF, PP = (a.ravel() for a in np.meshgrid(T, phi, P, indexing="ij"))
    sel = slice(rank, None, world)
    return TT[sel], PP[sel], ch4_air_Y(mech, FF[sel])


def hcci_block():
    """The hcciengine golden's cylinder (hcciengine.py:117-157): CKMI_ENG_* block (include/ckmi.h)."""
    ab = np.pi * 12.065 ** 2 / 4
    e = np.zeros(20)
    e[:7] = [-142.0, 1000.0, 16.5, 12.065, 14.005, 26.0093 / 7.0025, -0.5]
    e[7:12] = [1.0, 0.035, 0.71, 0.0, 400.0]
    e[12:16] = [2.28, 0.308, 3.24, 0.0]
    e[16:18] = [123.5 / ab, 124.75 / ab]
    return e


def model_line(kind, dm, dev, mech, ops, world, rank, args):
    """Plug-flow tubes (problem 3) or HCCI cylinders (problem 4) on the FP64-inverse wave kernel, one
    timed launch of a fixed total over the ranks.  flops count the batch-reactor RHS / Jacobian / LU
    work only (the engine's transport terms and the tube's rho / G scaling are not counted)."""
    from pychemkin_amd import transport as trn

    total = 16 ** 3 if kind == "pfr" else 16 ** 3 * 4
    if kind == "pfr":  # configs[2]-like tubes: 1 cm at 1 cm/s inlet velocity = 1 s of residence
        T0, P0, Y0 = model_sweep(mech, world, rank, total, 1100.0, 1700.0, P_ATM, 100 * P_ATM, 0.5, 2.0)
        cfg = _native.make_cfg(**RUN)
        orc_run = RUN
        workload = (f"plug-flow tubes: GRI-3.0 CH4/air, {total} tubes in total (16 T0 1100-1700 K x 16 phi x 16 P "
                    "1-100 atm), 1 cm at 1 cm/s, momentum equation on, TIFP")
    else:
        T0, P0, Y0 = model_sweep(mech, world, rank, total, 420.0, 520.0, 1.0 * P_ATM, 2.0 * P_ATM, 0.3, 1.0)
        text = open(os.path.join(ROOT, "data", "grimech30_transport.dat")).read()
        params = trn.species_params(trn.parse_transport_text(text), mech.species)
        th = mech.to_tables()["thermo"]
        fits = np.hstack([trn.viscosity_fits(mech.wt, params), trn.conductivity_fits(mech.wt, params, th)])
        tran = torch.tensor(fits, dtype=torch.float64, device=dev)
        # NNEG as the reference's HCCI example sets it (hcciengine.py:173): without it 3-4 of the 15,625
        # cylinders stall in the expansion stroke on the GPU
        run = dict(RUN, t_end=258.0 / 6000.0, nneg=True)
        cfg = _native.make_cfg(engine=hcci_block(), tran=tran, **run)
        orc_run = dict(run, engine=hcci_block(), tran=fits)
        workload = (f"HCCI cylinders: GRI-3.0 CH4/air, {round(total ** (1 / 3)) ** 3} in total (T_IVC 420-520 K x "
                    "phi 0.3-1 x P_IVC 1-2 atm), the hcciengine golden's engine, ICHX/Woschni wall heat, -142..116 CA, NNEG")
    code = 3 if kind == "pfr" else 4
    sh = Shard(dm, dev, T0, P0, Y0, np.full(len(T0), code, np.int32))
    sh.step(cfg, 0, min(sh.n, 256))
    tmax, kern_ms, res = timed(world, lambda: sh.step(cfg), 1)
    stats = res["stats"].cpu().numpy()
    tau = res["tau"].cpu().numpy()
    # TIFP always finds a largest dT/dt (compression heating, too): a tube or cylinder counts as ignited
    # only when it ends at least 200 K above its initial temperature
    Tend = res["T"].cpu().numpy()
    not_ign = int(((tau <= 0) | (Tend < np.asarray(T0) + 200.0)).sum())
    tot = torch.tensor([sh.n], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot)
    tot = int(tot.item())
    unit = "tubes/s" if kind == "pfr" else "cylinders/s"
    del sh, res
    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_reactor_baseline(mech, np.asarray(T0), np.asarray(P0), np.asarray(Y0), np.full(len(T0), code, np.int32),
                                   tau, args.cpu_seconds_secondary, args.cpu_sample, single=True, run=orc_run)
        cpu["unit"] = unit
    return {"metric": f"{'plug-flow reactor' if kind == 'pfr' else 'engine cycle'} integrations/sec ({workload})",
            "value": tot / tmax, "unit": unit, "total": tot, "per_gpu": len(T0), "seconds": tmax, "scaling": "strong",
            "failed": int((stats[:, 6] != 0).sum()), "runaway": int((stats[:, 6] == 4).sum()), "not_ignited": not_ign,
            "solver": solver_summary(stats),
            "roofline": reactor_roofline(ops, stats, float(np.mean(kern_ms)) / 1e3, "reactor_kernel<54, false, true>",
                                         f"reactor_{kind}", len(T0)),
            "cpu_baseline": cpu}


def c1_line(args):
    """configs[0] latency: one reactor through the drop-in API, the way a PyChemkin user runs it."""
    import pychemkin_amd as ck
    from pychemkin_amd.batch import BatchSweep

    chem = ck.Chemistry(chem=os.path.join(ROOT, "data", "grimech30_chem.inp"),
                        therm=os.path.join(ROOT, "data", "grimech30_thermo.dat"), label="GRI 3.0")
    chem.preprocess()
    fuel = ck.Mixture(chem)
    fuel.X = [("CH4", 1.0)]
    air = ck.Mixture(chem)
    air.X = [("O2", 0.21), ("N2", 0.79)]
    mix = ck.Mixture(chem)
    mix.X_by_Equivalence_Ratio(chem, fuel.X, air.X, np.zeros(chem.KK), ["CO2", "H2O", "N2"], 1.0)
    mix.temperature = 1200.0
    mix.pressure = P_ATM
    r = ck.GivenPressureBatchReactor_EnergyConservation(mix, label="c1")
    r.volume = 1.0
    r.time = RUN["t_end"]
    r.tolerances = (RUN["atol"], RUN["rtol"])
    r.set_ignition_delay(method="T_inflection")
    assert r.run() == 0  # warm-up: device mechanism, code objects, JIT
    lat = []
    for _ in range(7):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rc = r.run()
        tau = r.get_ignition_delay()
        lat.append((time.perf_counter() - t0) * 1e3)
        assert rc == 0
    stats = r.solver_statistics
    from oracle.oracle import Oracle  # noqa: E402  (cpu_baseline leg only)

    orc = Oracle(chem.mechanism)
    cl = []
    for _ in range(3):
        t0 = time.perf_counter()
        ro, _ = orc.reactor(mix.temperature, mix.pressure, 1.0, mix.Y, problem=1, **RUN)
        cl.append((time.perf_counter() - t0) * 1e3)
    # the reference's serial loop (ignitiondelay.py:127-144): one run() per condition, T0 += 20 K
    temps = 1200.0 + 20.0 * np.arange(20)
    t0 = time.perf_counter()
    taus = []
    for T in temps:
        r.temperature = T
        assert r.run() == 0
        taus.append(r.get_ignition_delay())
    loop_s = time.perf_counter() - t0
    sweep = BatchSweep(chem, problem="CONP", energy="ENERGY", t_end=RUN["t_end"], atol=RUN["atol"], rtol=RUN["rtol"],
                       ignition="T_inflection", devices=[torch.cuda.current_device()])
    sweep.run(temps[:2], P_ATM, Y0=mix.Y)  # warm-up
    t0 = time.perf_counter()
    br = sweep.run(temps, P_ATM, Y0=mix.Y)
    batch_s = time.perf_counter() - t0
    return {"metric": "single-reactor latency (configs[0]: GRI-3.0 CONP CH4/air phi 1, 1200 K, 1 atm, t_end 1 s, TIFP, "
                      "1e-10/1e-8, drop-in run())",
            "latency_ms": float(np.median(lat)), "latency_ms_all": lat, "tau_ms": tau, "unit": "ms",
            "higher_is_better": False, "solver": {k: int(v) for k, v in stats.items()},
            "cpu_baseline": {"value": float(np.median(cl)), "unit": "ms", "cores": 1, "kind": "port",
                             "sample": "the same reactor, oracle C restatement, 1 thread, median of 3",
                             "tau_rel_diff_vs_gpu": abs(ro.tau * 1e3 / tau - 1), "nst": ro.nst, "nfe": ro.nfe,
                             "nlu": ro.nlu},
            "serial_loop_20": {"seconds": loop_s, "per_run_ms": loop_s / 20 * 1e3,
                               "pattern": "ignitiondelay.py:127-144: reactor.temperature = T; run(); get_ignition_delay()"},
            "batch_20": {"seconds": batch_s, "speedup_vs_serial_loop": loop_s / batch_s,
                         "tau_max_rel_diff_vs_loop": float(np.max(np.abs(br.tau * 1e3 / np.asarray(taus) - 1)))}}


def _free_port():
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as so:
        so.bind(("127.0.0.1", 0))
        return so.getsockname()[1]


def launch_ranks(n, argv, visible=None):
    """bench.py --gpus N run directly: start N rank processes (children, never exec) on one node and
    return (worst exit status, rank 0's stdout).  Called before anything initialises a GPU
    (torch.cuda.device_count() does not); N must not exceed the visible devices."""
    if visible is not None and n > visible:
        raise SystemExit(f"bench.py: --gpus {n} but only {visible} GPU(s) are visible")
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + argv, env=env,
                                      stdout=subprocess.PIPE if r == 0 else subprocess.DEVNULL))
    out0 = procs[0].communicate()[0].decode()
    rcs = [procs[0].returncode] + [p.wait() for p in procs[1:]]
    return max(rcs, key=abs), out0


def plan(world, rank):
    """--plan: the sharding and the timing protocol of a run without a GPU (gloo): every rank builds
    its shard of the headline sweep, 'runs' for a rank-dependent time between the same barriers, and
    rank 0 reports the shard sizes, whether the shards are disjoint and complete, and the
    max-over-ranks time that value would be computed from."""
    if world > 1:
        dist.init_process_group(backend="gloo", init_method="env://")
    idx = torch.as_tensor(sweep_index(world, rank))
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    time.sleep(0.05 * (rank + 1))
    if world > 1:
        dist.barrier()
    elapsed = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    mine = elapsed.clone()
    if world > 1:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
        sizes = [torch.zeros(1, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(sizes, torch.tensor([idx.numel()]))
        allidx = [torch.zeros(int(k.item()), dtype=idx.dtype) for k in sizes]
        dist.all_gather(allidx, idx)
        times = [torch.zeros(1, dtype=torch.float64) for _ in range(world)]
        dist.all_gather(times, mine)
    else:
        allidx, times = [idx], [mine]
    if rank == 0:
        cat = torch.cat(allidx)
        total = 65536 * world
        print(json.dumps({"plan": True, "n_ranks": world, "shard_sizes": [int(a.numel()) for a in allidx],
                          "disjoint": int(torch.unique(cat).numel()) == int(cat.numel()),
                          "complete": int(torch.unique(cat).numel()) == total and int(cat.min()) == 0
                          and int(cat.max()) == total - 1,
                          "rank_seconds": [float(t.item()) for t in times], "max_seconds": float(elapsed.item())}),
              flush=True)
    if world > 1:
        dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=None, help="GPUs of this node (default: WORLD_SIZE, else 1)")
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--reactors", type=int, default=0, help="override the headline reactors per GPU (0 = full 65,536)")
    ap.add_argument("--sub-reactors", type=int, default=0, help="cap the c4 / c5 shards (0 = full sweeps)")
    ap.add_argument("--lines", default="c1,c3,c4,c5,rop,lu,rop161,ropext,pfr,hcci",
                    help="comma list of: c1, c3 (headline, always run), c4, c5, rop, lu, rop161, ropext, pfr, hcci")
    ap.add_argument("--rop-states", type=int, default=10_000_000)
    ap.add_argument("--lu-systems", type=int, default=16384)
    ap.add_argument("--big-states", type=int, default=1_000_000)
    ap.add_argument("--cpu-sample", type=int, default=16384, help="max reactors in a CPU-baseline sample (0 = skip)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline budget of the headline")
    ap.add_argument("--cpu-seconds-secondary", type=float, default=6.0, help="CPU-baseline budget of c4 / c5")
    ap.add_argument("--plan", action="store_true", help="print the shard layout / timing protocol (no GPU)")
    args = ap.parse_args()
    lines = set(args.lines.split(","))

    if "WORLD_SIZE" not in os.environ and (args.gpus or 1) > 1:  # be the launcher (no GPU touched yet)
        visible = None if args.plan else torch.cuda.device_count()
        rc, out0 = launch_ranks(args.gpus, sys.argv[1:], visible)
        sys.stdout.write(out0)
        sys.stdout.flush()
        raise SystemExit(rc)
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus is not None and args.gpus != world:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE is {world}")
    if args.plan:
        plan(world, rank)
        return
    if world > 1:
        dist.init_process_group(backend="nccl", init_method="env://")
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)

    mech = mechanism()
    tables = mech.to_tables()
    ops = count_ops(tables)
    dm = _native.DeviceMechanism(tables, device=dev)

    # ---- headline: configs[2]
    T0, P0, Y0, prob = sweep(mech, world, rank)
    if args.reactors:
        T0, P0, Y0, prob = T0[: args.reactors], P0[: args.reactors], Y0[: args.reactors], prob[: args.reactors]
    sh = Shard(dm, dev, T0, P0, Y0, prob)
    n = sh.n
    cfg = _native.make_cfg(**RUN)
    for _ in range(args.warmup):
        sh.step(cfg)
    tmax, kern_ms, res = timed(world, lambda: sh.step(cfg), args.steps)
    stats = res["stats"].cpu().numpy()
    tau = res["tau"].cpu().numpy()
    kern_s = float(np.mean(kern_ms)) / 1e3
    value = n * world * args.steps / tmax

    # PCIe-inclusive rate (reported beside value, never as value): host numpy inputs -> H2D ->
    # one launch -> D2H of tau, T, P, V, Y, stats, on this rank
    torch.cuda.synchronize()
    tp = time.perf_counter()
    rp = dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0)
    host_out = {k: v.cpu().numpy() for k, v in rp.items() if not k.startswith("_")}
    torch.cuda.synchronize()
    pcie_s = time.perf_counter() - tp
    pcie = {"reactors_per_s": n / pcie_s, "seconds": pcie_s, "vs_value": (n / pcie_s) / (value / world),
            "bytes_h2d": int(T0.nbytes + P0.nbytes + Y0.nbytes + prob.nbytes + 8 * n),
            "bytes_d2h": int(sum(a.nbytes for a in host_out.values()))}
    del rp, host_out

    cpu = None
    if rank == 0 and world == 1 and args.cpu_sample > 0:
        cpu = cpu_reactor_baseline(mech, T0, P0, Y0, prob, tau, args.cpu_seconds, args.cpu_sample)
    del sh, res

    c4 = c5 = rop = lu = rop_big = None
    if "c4" in lines:
        c4 = secondary_sweep("c4", dm, dev, mech, ops, sweep_c4, world, rank, args, "reactor_kernel<54>", "reactor_c4",
                             "configs[3]: GRI-3.0 CH4/air 128 T0 x 64 phi x 64 P x {CONP, CONV} = 2^20 reactors in total",
                             "strong")
    if "c5" in lines:
        bm = big_mechanism()
        bops = count_ops(bm.to_tables())
        bdm = _native.DeviceMechanism(bm.to_tables(), device=dev)
        c5 = secondary_sweep("c5", bdm, dev, bm, bops, sweep_c5, world, rank, args, "big_reactor_kernel<11>",
                             "big_reactor_c5",
                             "configs[4] stand-in: 161-species GRI-3.0 + 108-tracer mechanism (no n-heptane mechanism "
                             "offline; parity with Chemkin unpinned), 64 T0 x 64 phi x 64 P = 262,144 CONP reactors in "
                             "total", "strong")
        c5["mechanism"] = f"data/gri30_tracer161 (KK = {bm.KK}, II = {bm.II}, n = {bm.KK + 1})"
        bdm.close()
    if "rop" in lines and args.rop_states > 0:
        rop = rop_line(dev, mech, ops, args.rop_states, rank, world, args.cpu_sample)
    if "lu" in lines and rank == 0 and args.lu_systems > 0:
        lu = lu_line(dev, args.lu_systems, 161, args.cpu_sample if world == 1 else 0)
    if "rop161" in lines and rank == 0 and args.big_states > 0:
        bm = big_mechanism()
        rop_big = rop_line(dev, bm, count_ops(bm.to_tables()), args.big_states, rank, world, args.cpu_sample,
                           kernel_name="rop_kernel<0,3>", traffic_key="rop_161sp",
                           label=f"synthetic GRI-3.0 + tracers, KK = {bm.KK}, II = {bm.II}")
    rop_ext = None
    if "ropext" in lines and rank == 0 and args.big_states > 0:
        # every reaction form on the specialised kernel: PLOG, HIGH, FORD / RORD, fractional and wide
        # reactions (count_ops prices a PLOG / general reaction like an Arrhenius one: a lower bound)
        em = Mechanism.from_files(os.path.join(ROOT, "data", "gri30_tracer161_ext_chem.inp"),
                                  os.path.join(ROOT, "data", "gri30_tracer161_thermo.dat"))
        rop_ext = rop_line(dev, em, count_ops(em.to_tables()), args.big_states, rank, world, args.cpu_sample,
                           kernel_name="rop_kernel<0,3,true>", traffic_key="rop_ext",
                           label=f"data/gri30_tracer161_ext (PLOG, HIGH, FORD/RORD, fractional, wide), KK = {em.KK}, "
                                 f"II = {em.II}")

    c1 = c1_line(args) if "c1" in lines and rank == 0 else None
    pfr = model_line("pfr", dm, dev, mech, ops, world, rank, args) if "pfr" in lines else None
    hcci = model_line("hcci", dm, dev, mech, ops, world, rank, args) if "hcci" in lines else None

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
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic",
            "config": {"workload": "configs[2]: GRI-3.0 CONP CH4/air ignition sweep 64 T0 x 32 phi x 32 P per GPU",
                       "reactors_per_gpu": n, "t_end_s": RUN["t_end"], "atol": RUN["atol"], "rtol": RUN["rtol"],
                       "ignition": "TIFP", "parallelism": f"shard-by-condition x{world}"},
            "value_excludes_pcie": True,
            "reactors_per_min": value * 60.0,
            "failed_reactors": int((stats[:, 6] != 0).sum()),
            "not_ignited": int((tau <= 0).sum()),
            "solver": solver_summary(stats),
            "roofline": reactor_roofline(ops, stats, kern_s, "reactor_kernel<54>", "reactor", n),
            "cpu_baseline": cpu,
            "pcie_inclusive": pcie,
            "c1": c1,
            "c4": c4,
            "c5": c5,
            "rop": rop,
            "lu": lu,
            "rop_161sp": rop_big,
            "rop_ext161": rop_ext,
            "pfr": pfr,
            "hcci": hcci,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
