"""The BASELINE.json configurations at their full sizes, through the C ABI on the GPU.

configs[2]: the 65,536-reactor CONP ignition sweep (bench.sweep, one launch, ~1.2 s);
configs[3]: the 2^20-reactor CONP + CONV sweep (bench.sweep_c4, one launch, ~19 s);
configs[4]: the 262,144-reactor sweep of the 161-species stand-in (bench.sweep_c5) -- a strided
            1/8 sample here (~10 s; the full sweep is the bench's c5 line).
Each is checked by size-independent properties (every reactor succeeds and ignites, mass and
elements are conserved, ignition delay falls with T0) and against the oracle on a strided
subsample: tau within 1e-4 relative, final T within 1e-4 (the north_star bar is 0.5 % / 1e-4).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _drift(mech, Y0, Y):
    ncf = mech.ncf.astype(float)
    e0 = (Y0 / mech.wt) @ ncf.T
    e1 = (Y / mech.wt) @ ncf.T
    return np.max(np.abs(e1 - e0) / np.max(e0, axis=1, keepdims=True), axis=1)


def _conservation(mech, Y0, Y, tol=2e-9):
    """Mass closes to 1e-7 and elements are conserved to `tol` in every reactor.  The integrators hold
    element conservation to 0.1 rtol (1e-9 at the bench's rtol 1e-8): an accepted step whose element
    content has drifted further is projected back (include/ckmi.h no_elem_proj, oracle elem_project);
    below that the drift is the chaotic residue of the Newton convergence of each step (round 5, without
    the projection: a tail up to 3e-7 on the GPU, 13x the oracle's on some configs[4] reactors).  The
    final state is interpolated inside the last step, hence the bar of 0.2 rtol."""
    assert np.allclose(Y.sum(axis=1), 1.0, atol=1e-7)
    d = _drift(mech, Y0, Y)
    assert d.max() < tol
    return d


def _oracle_sample(mech, T0, P0, Y0, prob, res, nsample, d_gpu, threads=16):
    """tau and final T of a strided subsample against the oracle (1e-4), and the element-drift
    distribution of the GPU on that subsample against the oracle's (90th percentile within 10x).
    Returns the oracle's drifts."""
    from oracle.oracle import Oracle

    import bench

    idx = np.linspace(0, T0.size - 1, nsample).astype(np.int64)
    orc = Oracle(mech)
    nfail, ref, Yo = orc.reactor_batch(T0[idx], P0[idx], Y0[idx], problem=prob[idx], V0=np.ones(idx.size),
                                       nthreads=threads, **bench.RUN)
    assert nfail == 0
    tau_o = np.array([r.tau for r in ref])
    T_o = np.array([r.T for r in ref])
    assert np.max(np.abs(res["tau"][idx] / tau_o - 1)) < 1e-4
    assert np.max(np.abs(res["T"][idx] / T_o - 1)) < 1e-4
    d_o = _drift(mech, Y0[idx], np.asarray(Yo))
    assert np.percentile(d_gpu[idx], 90) <= 10.0 * np.percentile(d_o, 90) + 1e-11
    return d_o


def _run(dm, T0, P0, Y0, prob):
    from pychemkin_amd import _native

    import bench

    res = dm.reactor_run(_native.make_cfg(**bench.RUN), prob, T0, P0, np.ones(T0.size), Y0)
    return {k: v.cpu().numpy() for k, v in res.items() if not k.startswith("_")}


def test_configs2_full_sweep(tables, mech):
    """configs[2]: 64 T0 x 32 phi x 32 P = 65,536 CONP reactors in one launch."""
    from pychemkin_amd import _native

    import bench

    dm = _native.DeviceMechanism(tables)
    T0, P0, Y0, prob = bench.sweep(mech, 1, 0)
    assert T0.size == 65536
    res = _run(dm, T0, P0, Y0, prob)
    assert np.all(res["stats"][:, 6] == 0)
    assert np.all(res["tau"] > 0) and np.all(res["tau"] < 1.0)
    assert np.all(res["T"] > T0 + 300.0)
    d = _conservation(mech, Y0, res["Y"])
    tau = res["tau"].reshape(64, 32, 32)  # (T0, phi, P)
    assert np.all(np.diff(np.log(tau), axis=0) < 0)  # hotter ignites sooner (no NTC for CH4 at 1100-1700 K)
    _oracle_sample(mech, T0, P0, Y0, prob, res, 256, d)


def test_configs3_full_sweep(tables, mech):
    """configs[3]: 128 T0 x 64 phi x 64 P x {CONP, CONV} = 2^20 reactors in one launch."""
    from pychemkin_amd import _native

    import bench

    dm = _native.DeviceMechanism(tables)
    T0, P0, Y0, prob = bench.sweep_c4(mech, 1, 0)
    assert T0.size == 2 ** 20
    res = _run(dm, T0, P0, Y0, prob)
    assert np.all(res["stats"][:, 6] == 0)
    assert np.all(res["tau"] > 0) and np.all(res["tau"] < 1.0)
    d = _conservation(mech, Y0, res["Y"])
    conp, conv = prob == 1, prob == 2
    # CONP keeps P, CONV keeps V (V0 = 1) and raises P with the temperature
    assert np.allclose(res["P"][conp], P0[conp], rtol=1e-12)
    assert np.allclose(res["V"][conv], 1.0, rtol=1e-12) and np.all(res["P"][conv] > P0[conv])
    # the same condition ignites sooner at constant volume (pressure rises with heat release)
    assert np.all(res["tau"][conv] <= res["tau"][conp] * (1 + 1e-3))
    tau = res["tau"][conp].reshape(128, 64, 64)
    assert np.all(np.diff(np.log(tau), axis=0) < 0)
    _oracle_sample(mech, T0, P0, Y0, prob, res, 256, d)


def test_configs4_sample(big_mech):
    """configs[4] stand-in: every 8th reactor of the 262,144-reactor sweep (32,768 reactors) on the
    workgroup-per-reactor kernel."""
    from pychemkin_amd import _native

    import bench

    dm = _native.DeviceMechanism(big_mech.to_tables())
    T0, P0, Y0, prob = bench.sweep_c5(big_mech, 8, 3)
    assert T0.size == 32768
    res = _run(dm, T0, P0, Y0, prob)
    assert np.all(res["stats"][:, 6] == 0)
    assert np.all(res["tau"] > 0) and np.all(res["tau"] < 1.0)
    assert np.all(res["T"] > T0 + 300.0)
    d = _conservation(big_mech, Y0, res["Y"])
    # the drift distribution of all 32,768 against the oracle's on a 1,024-reactor strided subsample of the
    # same sweep: 99th / 99.9th percentile and maximum within 2x (round-5 verdict item 1; the round-5
    # single-reactor envelope bar broke on legitimate summation-order changes of the Jacobian)
    d_o = _oracle_sample(big_mech, T0, P0, Y0, prob, res, 1024, d)
    q_g = [np.percentile(d, 99), np.percentile(d, 99.9), d.max()]
    q_o = [np.percentile(d_o, 99), np.percentile(d_o, 99.9), d_o.max()]
    print("configs[4] sample drift p99 / p99.9 / max: GPU", ["%.3e" % x for x in q_g], "oracle",
          ["%.3e" % x for x in q_o])
    assert all(g <= 2.0 * o + 1e-12 for g, o in zip(q_g, q_o))
    assert d.max() <= 2.0 * np.percentile(d_o, 99.9) + 1e-12
