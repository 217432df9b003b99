"""Batched reactor sweeps: the GPU-native replacement of the reference's serial run() loop.

The reference integrates a sweep one reactor at a time from Python
(tests/integration_tests/ignitiondelay.py:127-144, sensitivity.py:141-160).  ``BatchSweep``
takes the whole set of initial conditions, shards it by condition across the visible GPUs
(strided, so that cheap and expensive conditions are spread evenly) and
runs one ckmi_reactor_run launch per GPU.  There is no exchange between shards; results are
gathered on the host.
"""
from __future__ import annotations

from dataclasses import dataclass
from typing import Dict, List, Optional, Sequence

import numpy as np

from . import _native
from .chemistry import Chemistry
from .mixture import Mixture

PROBLEMS = {"CONP": 1, "CONV": 2, 1: 1, 2: 2}
ENERGIES = {"ENERGY": 1, "ENRG": 1, "GivenT": 2, "TGIV": 2, 1: 1, 2: 2}


@dataclass
class BatchResult:
    tau: np.ndarray          # ignition delay [s] (-1: not detected)
    T: np.ndarray            # final temperature [K]
    P: np.ndarray            # final pressure [dyn/cm2]
    V: np.ndarray            # final volume [cm3]
    Y: np.ndarray            # final mass fractions [n, KK]
    stats: np.ndarray        # [n, 8] int32 solver statistics (see _native.STAT_NAMES)
    wt: np.ndarray

    @property
    def ignition_delay_ms(self) -> np.ndarray:
        return self.tau * 1.0e3

    @property
    def status(self) -> np.ndarray:
        return self.stats[:, 6]

    @property
    def X(self) -> np.ndarray:
        x = self.Y / self.wt
        return x / x.sum(axis=1, keepdims=True)

    def statistics(self) -> Dict[str, np.ndarray]:
        return {k: self.stats[:, i] for i, k in enumerate(_native.STAT_NAMES)}


class BatchSweep:
    """Run many independent batch reactors that share one configuration."""

    def __init__(self, chem: Chemistry, problem="CONP", energy="ENERGY", t_end: float = 1.0, atol: float = 1.0e-12,
                 rtol: float = 1.0e-6, ignition: Optional[str] = "T_inflection", ign_val: float = 0.0,
                 ign_target: str = "", nneg: bool = False, h0: float = 0.0, hmax: float = 0.0,
                 ign_stop: bool = False, profile=None, max_steps: int = 0, devices: Optional[Sequence[int]] = None,
                 **keywords):
        """keywords: the remaining typed reactor keywords of _native.make_cfg -- gfac (GFAC), qloss (QLOS,
        cal/s), htc (HTC), areaq (AREAQ), tamb (TAMB), prof_kind (1: `profile` is TPRO), profile2 /
        prof2_kind (QPRO / AEXT), asteps / avar / avalue (adaptive solution points)."""
        self.chem = chem
        self.problem = PROBLEMS[problem]
        sp = chem.get_specindex(ign_target) if ignition == "Species_peak" else 0
        self.cfg = _native.make_cfg(energy=ENERGIES[energy], t_end=t_end, atol=max(atol, 1e-20),
                                    rtol=max(rtol, 1e-12), h0=h0, hmax=hmax, nneg=nneg, ign_mode=ignition,
                                    ign_val=ign_val, ign_species=sp, ign_stop=ign_stop, max_steps=max_steps,
                                    profile=profile, **keywords)
        self.devices = list(devices) if devices is not None else None

    def _devices(self) -> List[int]:
        import torch

        if self.devices is not None:
            return self.devices
        return list(range(torch.cuda.device_count()))

    def run(self, T0, P0, X0=None, Y0=None, V0=None, problem=None, afac_rxn=None, afac=None) -> BatchResult:
        """Integrate reactors i = 0..n-1 from (T0[i], P0[i], X0[i] or Y0[i], V0[i]).

        afac_rxn[i] / afac[i]: reactor i runs with the A factor of reaction afac_rxn[i] (0-based,
        -1 none) multiplied by afac[i] -- the batched form of set_reaction_AFactor + run()."""
        import torch

        T0 = np.asarray(T0, dtype=np.float64).reshape(-1)
        n = T0.size
        P0 = np.broadcast_to(np.asarray(P0, dtype=np.float64), (n,)).copy()
        V0 = np.ones(n) if V0 is None else np.broadcast_to(np.asarray(V0, dtype=np.float64), (n,)).copy()
        wt = self.chem.WT
        if Y0 is None:
            if X0 is None:
                raise ValueError("X0 or Y0 is required")
            X = np.atleast_2d(np.asarray(X0, dtype=np.float64))
            X = np.broadcast_to(X, (n, wt.size))
            Y = X * wt
            Y0 = Y / Y.sum(axis=1, keepdims=True)
        Y0 = np.ascontiguousarray(np.broadcast_to(np.atleast_2d(np.asarray(Y0, dtype=np.float64)), (n, wt.size)))
        if problem is None:
            prob = np.full(n, self.problem, np.int32)
        else:
            prob = np.asarray([PROBLEMS[p] for p in np.broadcast_to(np.asarray(problem, dtype=object), (n,))], np.int32)
        devs = self._devices()
        if not devs:
            raise _native.NativeError("no ROCm GPU visible: BatchSweep requires at least one MI355X")
        shards = [np.arange(r, n, len(devs)) for r in range(len(devs))]
        pending = []
        for d, idx in zip(devs, shards):
            if idx.size == 0:
                continue
            dm = self.chem.device_mechanism(d)
            pert = {}
            if afac_rxn is not None:
                pert = dict(afac_rxn=np.asarray(afac_rxn, np.int32).reshape(-1)[idx],
                            afac=np.broadcast_to(np.asarray(afac, np.float64), (n,))[idx])
            with torch.cuda.device(d):
                res = dm.reactor_run(self.cfg, prob[idx], T0[idx], P0[idx], V0[idx], Y0[idx], **pert)
            pending.append((idx, res))
        out = BatchResult(tau=np.empty(n), T=np.empty(n), P=np.empty(n), V=np.empty(n), Y=np.empty((n, wt.size)),
                          stats=np.empty((n, _native.NSTAT), np.int32), wt=wt)
        for idx, res in pending:
            out.tau[idx] = res["tau"].cpu().numpy()
            out.T[idx] = res["T"].cpu().numpy()
            out.P[idx] = res["P"].cpu().numpy()
            out.V[idx] = res["V"].cpu().numpy()
            out.Y[idx] = res["Y"].cpu().numpy()
            out.stats[idx] = res["stats"].cpu().numpy()
        return out

    def run_mixtures(self, mixtures: Sequence[Mixture], V0=None, problem=None) -> BatchResult:
        T0 = [m.temperature for m in mixtures]
        P0 = [m.pressure for m in mixtures]
        Y0 = np.stack([m.Y for m in mixtures])
        return self.run(T0, P0, Y0=Y0, V0=V0, problem=problem)


def afactor_sensitivity(chem: Chemistry, mixture: Mixture, factor: float = 1.001, reactions: Optional[Sequence[int]] = None,
                        volume: float = 1.0, **sweep_kw) -> Dict[str, np.ndarray]:
    """Brute-force A-factor sensitivity of the ignition delay (reference sensitivity.py:122-160).

    The reference perturbs one reaction's A by `factor` and re-runs the reactor serially (326
    native runs for GRI-3.0).  Here the nominal reactor and every perturbed one are reactors of
    ONE batch (per-reactor A multiplier, ckmi_reactor_run_ex), sharded over the visible GPUs.
    Returns S_i = (tau_i - tau_0) / (factor - 1) [s] per 0-based reaction, tau_0 [s], and the
    per-reactor status.
    """
    II = chem.IIGas
    rx = np.arange(II) if reactions is None else np.asarray(list(reactions), dtype=np.int64)
    if np.any(rx < 0) or np.any(rx >= II):
        raise ValueError("reaction indices must be 0-based and < IIGas")
    n = rx.size + 1
    sweep = BatchSweep(chem, **sweep_kw)
    afac_rxn = np.concatenate([[-1], rx]).astype(np.int32)
    r = sweep.run(np.full(n, mixture.temperature), np.full(n, mixture.pressure), Y0=np.tile(mixture.Y, (n, 1)),
                  V0=np.full(n, volume), afac_rxn=afac_rxn, afac=np.full(n, float(factor)))
    tau0 = float(r.tau[0])
    sens = (r.tau[1:] - tau0) / (factor - 1.0)
    return {"reactions": rx, "sensitivity": sens, "tau0": tau0, "status": r.status.copy()}
