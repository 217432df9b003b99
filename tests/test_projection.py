"""The corrector's element projection (oracle/ckoracle.c elem_project, ckmi_reactor.hpp elem_project_wave,
ckmi_big.hip elem_project_big): the oracle on CPU, both device kernels on the GPU."""
import numpy as np
import pytest


def _drift(mech, Y0, Y):
    ncf = mech.ncf.astype(float)
    e0 = (Y0 / mech.wt) @ ncf.T
    e1 = (Y / mech.wt) @ ncf.T
    return np.max(np.abs(e1 - e0) / np.max(e0, axis=1, keepdims=True), axis=1)


def _oracle_runs(mech, T0, P0, Y0, prob, proj):
    import bench
    from oracle.oracle import Oracle

    nf, res, Ye = Oracle(mech).reactor_batch(T0, P0, Y0, problem=prob, V0=np.ones(T0.size), nthreads=8,
                                             elem_proj=proj, **bench.RUN)
    assert nf == 0
    return np.array([r.tau for r in res]), np.array([r.nst for r in res]), Ye


def test_oracle_projection_untriggered_is_bitwise_unconstrained(mech):
    """GRI-3.0 at the bench tolerances: the oracle's drift never reaches 0.1 rtol, so the projection never
    acts and the results are bitwise those of the unconstrained BDF (the sensitivity golden's premise)."""
    import bench

    T0, P0, Y0, prob = bench.sweep(mech, 1, 0)
    idx = np.linspace(0, T0.size - 1, 24).astype(np.int64)
    on = _oracle_runs(mech, T0[idx], P0[idx], Y0[idx], prob[idx], True)
    off = _oracle_runs(mech, T0[idx], P0[idx], Y0[idx], prob[idx], False)
    assert np.array_equal(on[0], off[0]) and np.array_equal(on[1], off[1]) and np.array_equal(on[2], off[2])


def test_oracle_projection_bounds_drift(big_mech):
    """configs[4] stand-in: with the projection every reactor ends within 0.2 rtol of its initial element
    content (the check holds 0.1 rtol at every accepted step; the end state is interpolated inside the last
    step), at the same ignition delays (the projection moves each species by a relative ~1e-9)."""
    import bench

    T0, P0, Y0, prob = bench.sweep_c5(big_mech, 8, 3)
    idx = np.linspace(0, T0.size - 1, 24).astype(np.int64)
    tau_on, nst_on, Y_on = _oracle_runs(big_mech, T0[idx], P0[idx], Y0[idx], prob[idx], True)
    tau_off, nst_off, _ = _oracle_runs(big_mech, T0[idx], P0[idx], Y0[idx], prob[idx], False)
    d = _drift(big_mech, Y0[idx], Y_on)
    assert d.max() < 0.2 * bench.RUN["rtol"]
    assert np.max(np.abs(tau_on / tau_off - 1)) < 1e-6
    assert nst_on.mean() < 1.05 * nst_off.mean()


@pytest.mark.gpu
@pytest.mark.parametrize("big", [False, True])
def test_device_projection_on_off(mech, big_mech, big):
    """Both kernels with the projection on and off (cfg.no_elem_proj): on, every reactor of a strided sample
    stays within 0.2 rtol of its element content; off, the kernels are the unconstrained integrator (the
    round-5 drift tail); the ignition delays agree to 1e-5 either way."""
    import bench
    from pychemkin_amd import _native

    m = big_mech if big else mech
    T0, P0, Y0, prob = bench.sweep_c5(m, 8, 3) if big else bench.sweep(m, 1, 0)
    idx = np.linspace(0, T0.size - 1, 2048).astype(np.int64)
    dm = _native.DeviceMechanism(m.to_tables())
    out = {}
    for proj in (True, False):
        r = dm.reactor_run(_native.make_cfg(elem_proj=proj, **bench.RUN), prob[idx], T0[idx], P0[idx],
                           np.ones(idx.size), Y0[idx])
        r = {k: v.cpu().numpy() for k, v in r.items() if not k.startswith("_")}
        assert np.all(r["stats"][:, 6] == 0)
        out[proj] = (r["tau"], _drift(m, Y0[idx], r["Y"]))
    print("drift max with / without the projection: %.2e / %.2e" % (out[True][1].max(), out[False][1].max()))
    assert out[True][1].max() < 0.2 * bench.RUN["rtol"]
    assert np.max(np.abs(out[True][0] / out[False][0] - 1)) < 1e-5
