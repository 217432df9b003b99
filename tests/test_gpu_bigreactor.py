"""The workgroup-per-reactor integrator (ckmi_big.hip): batch reactors of mechanisms with more than
63 species, SURVEY.md §8(d) configs[4] (~160 species).

No ~160-species mechanism exists offline (parity with Chemkin unpinned at this size), so
the stand-in is the synthetic GRI-3.0 + 108-tracer mechanism (data/make_tracer_mechanism.py, KK =
161, n = 162) and the checker is the oracle's BDF (oracle/ckoracle.c, itself pinned by the GRI
goldens and checked against the numpy restatement on this mechanism).  Bar:
tau <= 1e-4 relative and final T <= 1e-4 on >= 16 reactors; major species rtol 1e-4.

The same kernel also runs GRI-3.0 when forced (ckmi_set_reactor_path(1)); there it must agree with
the wave-per-reactor kernel of ckmi.hip, which runs the identical algorithm.
"""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y

pytestmark = pytest.mark.gpu

MAJOR = ("CH4", "O2", "N2", "H2O", "CO2", "CO", "H2", "AX1")


def tracer_Y(mech, phi, frac=0.2):
    """CH4/air at phi with `frac` of the N2 replaced by the tracer AX1 (the stand-in's workload)."""
    phi = np.atleast_1d(np.asarray(phi, dtype=np.float64))
    X = np.zeros((phi.size, mech.KK))
    X[:, mech.species.index("CH4")] = phi
    X[:, mech.species.index("O2")] = 2.0
    X[:, mech.species.index("N2")] = 7.52 * (1.0 - frac)
    X[:, mech.species.index("AX1")] = 7.52 * frac
    Y = X * mech.wt
    return Y / Y.sum(axis=1, keepdims=True)


@pytest.fixture(scope="module")
def big(big_mech):
    from oracle.oracle import Oracle
    from pychemkin_amd import _native

    return big_mech, Oracle(big_mech), _native.DeviceMechanism(big_mech.to_tables())


RUN = dict(energy=1, t_end=0.02, atol=1e-10, rtol=1e-8, ign_mode="TIFP")


def _cases(n, seed):
    rng = np.random.default_rng(seed)
    T0 = rng.uniform(1250.0, 1700.0, n)
    P0 = P_ATM * rng.uniform(10.0, 60.0, n)
    phi = rng.uniform(0.5, 2.0, n)
    prob = np.where(np.arange(n) % 2 == 0, 1, 2).astype(np.int32)
    return T0, P0, phi, prob


def test_big_reactors_match_oracle(big):
    """16 CONP/CONV energy reactors of the 161-species stand-in against the oracle's BDF."""
    from pychemkin_amd import _native

    mech, orc, dm = big
    n = 16
    T0, P0, phi, prob = _cases(n, 11)
    Y0 = tracer_Y(mech, phi)
    res = dm.reactor_run(_native.make_cfg(**RUN), prob, T0, P0, np.ones(n), Y0)
    res = {k: v.cpu().numpy() for k, v in res.items() if not k.startswith("_")}
    nfail, ref, Yref = orc.reactor_batch(T0, P0, Y0, problem=prob, V0=np.ones(n), **RUN)
    assert nfail == 0
    for i in range(n):
        r = ref[i]
        assert res["stats"][i, 6] == 0, (i, res["stats"][i].tolist())
        assert r.tau > 0 and res["tau"][i] > 0
        assert abs(res["tau"][i] / r.tau - 1) < 1e-4, (i, res["tau"][i], r.tau)
        assert abs(res["T"][i] / r.T - 1) < 1e-4, (i, res["T"][i], r.T)
        for sp in MAJOR:
            k = mech.species.index(sp)
            assert abs(res["Y"][i, k] - Yref[i, k]) <= 1e-4 * max(abs(Yref[i, k]), 1e-3), (i, sp)
        # the tracer block is live: AX1 has spread over the chain
        assert res["Y"][i, mech.species.index("AX5")] > 0
        # mass is conserved
        assert abs(res["Y"][i].sum() - 1.0) < 1e-8
    # same integrator, but the Newton matrix is inverted by Gauss-Jordan (the oracle: LU) with fp32
    # pivot comparisons, so the step sequences drift apart at rounding level: counts stay close
    st = res["stats"]
    nst_o = np.array([r.nst for r in ref])
    assert np.all(np.abs(st[:, 0] - nst_o) <= 0.25 * nst_o)


def test_big_given_T_and_ign_stop(big):
    """Given-temperature CONP and DTIGN + IGN_STOP on the workgroup kernel vs the oracle."""
    from pychemkin_amd import _native

    mech, orc, dm = big
    n = 4
    T0, P0, phi, prob = _cases(n, 5)
    Y0 = tracer_Y(mech, phi)
    run = dict(energy=2, t_end=2e-3, atol=1e-12, rtol=1e-8, ign_mode=None)
    res = {k: v.cpu().numpy() for k, v in
           dm.reactor_run(_native.make_cfg(**run), prob, T0, P0, np.ones(n), Y0).items() if not k.startswith("_")}
    for i in range(n):
        r, Ye = orc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **run)
        assert res["stats"][i, 6] == 0 and r.status == 0
        assert res["T"][i] == T0[i]
        for sp in ("CH4", "O2", "CO", "H2O", "AX1", "AX2"):
            k = mech.species.index(sp)
            assert abs(res["Y"][i, k] - Ye[k]) <= 1e-4 * max(abs(Ye[k]), 1e-6), (i, sp)
    run = dict(energy=1, t_end=0.02, atol=1e-10, rtol=1e-8, ign_mode="DTIGN", ign_val=400.0, ign_stop=True)
    ts = np.linspace(0.0, 0.02, 21)
    res = dm.reactor_run(_native.make_cfg(**run), prob, T0, P0, np.ones(n), Y0, t_save=ts)
    res = {k: v.cpu().numpy() for k, v in res.items() if not k.startswith("_")}
    for i in range(n):
        r, _ = orc.reactor(T0[i], P0[i], 1.0, Y0[i], problem=int(prob[i]), **run)
        assert abs(res["tau"][i] / r.tau - 1) < 1e-4
        assert res["t_stop"][i] < 0.02 and res["T"][i] >= T0[i] + 400.0
        ys = res["y_save"][i]
        written = ts <= res["t_stop"][i]
        assert np.all(np.isfinite(ys[written])) and np.all(np.isnan(ys[~written]))


def test_workgroup_kernel_matches_wave_kernel_on_gri(tables, mech):
    """GRI-3.0 through both integrators: same algorithm, so tau / T agree far below the bar."""
    from pychemkin_amd import _native

    dm = _native.DeviceMechanism(tables)
    n = 64
    rng = np.random.default_rng(2)
    T0 = rng.uniform(1150.0, 1700.0, n)
    P0 = P_ATM * 10.0 ** rng.uniform(0.0, 2.0, n)
    Y0 = ch4_air_Y(mech, rng.uniform(0.5, 2.0, n))
    prob = np.where(np.arange(n) % 3 == 0, 2, 1).astype(np.int32)
    cfg = _native.make_cfg(energy=1, t_end=0.1, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    a = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0).items()
         if not k.startswith("_")}
    try:
        _native.set_reactor_path(1)
        b = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0).items()
             if not k.startswith("_")}
    finally:
        _native.set_reactor_path(0)
    assert np.all(a["stats"][:, 6] == 0) and np.all(b["stats"][:, 6] == 0)
    assert np.max(np.abs(a["tau"] / b["tau"] - 1)) < 1e-5
    assert np.max(np.abs(a["T"] / b["T"] - 1)) < 1e-7
    assert np.max(np.abs(a["Y"] - b["Y"])) < 1e-7


def test_workgroup_kernel_deterministic(big):
    """Bitwise-identical results on a re-run and under a permutation of the batch (no atomics
    whose order depends on wave timing)."""
    from pychemkin_amd import _native

    mech, _, dm = big
    n = 24
    T0, P0, phi, prob = _cases(n, 9)
    Y0 = tracer_Y(mech, phi)
    cfg = _native.make_cfg(**RUN)
    r1 = {k: v.cpu().numpy() for k, v in dm.reactor_run(cfg, prob, T0, P0, np.ones(n), Y0).items()
          if not k.startswith("_")}
    perm = np.random.default_rng(0).permutation(n)
    r2 = {k: v.cpu().numpy() for k, v in
          dm.reactor_run(cfg, prob[perm], T0[perm], P0[perm], np.ones(n), Y0[perm]).items() if not k.startswith("_")}
    for k in ("tau", "T", "P", "Y", "stats"):
        assert np.array_equal(r1[k][perm], r2[k]), k


def test_mechanism_creation_time(big_mech, tables):
    """Round-4 advice: ckmi_mech_create anneals the reaction-strip lane assignment on the host (400 proposals
    per slot, capped at 1024 slots' worth).  Creation of the GRI-3.0 and 161-species device tables, the
    annealing included, is timed and bounded."""
    import time

    from pychemkin_amd import _native

    for name, t in (("gri30", tables), ("tracer161", big_mech.to_tables())):
        t0 = time.perf_counter()
        dm = _native.DeviceMechanism(t)
        dt = time.perf_counter() - t0
        dm.close()
        print(f"ckmi_mech_create {name}: {dt * 1e3:.1f} ms")
        assert dt < 2.0
