"""Round-2 fixes on the device path: per-launch configurations, no host sync on the A-factor path,
and solutions of runs that stop early (IGN_STOP).

* Two launches with different configurations on ONE mechanism handle, on two streams, must give
  bitwise the results of the same launches run one after the other (the configuration used to
  live in one device buffer per handle, overwritten by every call).
* A DTIGN + IGN_STOP run followed by process_solution(): every solution row is finite, the
  trajectory ends at the stop time, and the reference semantics (the solution ends there,
  batchreactor.py:1335-1435) hold.
"""
import numpy as np
import pytest

from conftest import P_ATM, ch4_air_Y, h2_air_Y

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dm(tables):
    from pychemkin_amd import _native

    return _native.DeviceMechanism(tables)


def _inputs(mech, n, seed):
    rng = np.random.default_rng(seed)
    T0 = rng.uniform(1150.0, 1600.0, n)
    P0 = P_ATM * 10.0 ** rng.uniform(0.0, 1.5, n)
    Y0 = ch4_air_Y(mech, rng.uniform(0.6, 1.6, n))
    return T0, P0, Y0


def test_two_configs_two_streams_bitwise(dm, mech):
    import torch

    from pychemkin_amd import _native

    n = 512
    T0, P0, Y0 = _inputs(mech, n, 7)
    cfg_a = _native.make_cfg(energy=1, t_end=0.05, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    cfg_b = _native.make_cfg(energy=1, t_end=0.02, atol=1e-12, rtol=1e-6, ign_mode="DTIGN", ign_val=400.0)
    prob_a = np.ones(n, np.int32)
    prob_b = np.full(n, 2, np.int32)
    ser_a = {k: v.cpu() for k, v in dm.reactor_run(cfg_a, prob_a, T0, P0, np.ones(n), Y0).items()}
    ser_b = {k: v.cpu() for k, v in dm.reactor_run(cfg_b, prob_b, T0, P0, np.ones(n), Y0).items()}
    torch.cuda.synchronize()
    s1, s2 = torch.cuda.Stream(), torch.cuda.Stream()
    # both launches are enqueued before either finishes: each must read its own configuration
    with torch.cuda.stream(s1):
        ra = dm.reactor_run(cfg_a, prob_a, T0, P0, np.ones(n), Y0)
    with torch.cuda.stream(s2):
        rb = dm.reactor_run(cfg_b, prob_b, T0, P0, np.ones(n), Y0)
    torch.cuda.synchronize()
    for ser, par in ((ser_a, ra), (ser_b, rb)):
        for k in ("tau", "T", "P", "V", "Y", "stats", "t_stop"):
            assert torch.equal(ser[k], par[k].cpu()), k
    # the two configurations really differ in their results
    assert not torch.equal(ser_a["T"], ser_b["T"])


def test_afac_path_keeps_inputs_alive(dm, mech):
    """The A-factor inputs are referenced by the result (no stream synchronize in reactor_run)."""
    import torch

    from pychemkin_amd import _native

    n = 64
    T0, P0, Y0 = _inputs(mech, n, 3)
    cfg = _native.make_cfg(energy=1, t_end=0.05, atol=1e-10, rtol=1e-8, ign_mode="TIFP")
    rx = np.arange(n, dtype=np.int32) % 40
    res = dm.reactor_run(cfg, np.ones(n, np.int32), T0, P0, np.ones(n), Y0, afac_rxn=rx, afac=np.full(n, 2.0))
    assert "_inputs" in res
    # churn the caching allocator on the same stream while the launch may still be running
    junk = [torch.full((n,), -1.0, dtype=torch.float64, device=dm.device) for _ in range(8)]
    ref = dm.reactor_run(cfg, np.ones(n, np.int32), T0, P0, np.ones(n), Y0, afac_rxn=rx, afac=np.full(n, 2.0))
    torch.cuda.synchronize()
    del junk
    assert torch.equal(res["tau"].cpu(), ref["tau"].cpu())


def test_ign_stop_solution_ends_at_stop_time(chem, mech):
    import pychemkin_amd as ck

    mix = ck.Mixture(chem)
    mix.temperature = 1000.0
    mix.pressure = P_ATM
    mix.Y = h2_air_Y(mech)
    r = ck.GivenPressureBatchReactor_EnergyConservation(mix, label="stop")
    r.volume = 1.0
    r.time = 5.0e-4
    r.tolerances = (1.0e-20, 1.0e-8)
    r.force_nonnegative = True
    r.set_ignition_delay(method="T_rise", val=400.0)
    r.stop_after_ignition()
    assert r.run() == 0
    tau_ms = r.get_ignition_delay()
    assert 0.2 < tau_ms < 0.4
    r.process_solution()
    t = r.get_solution_variable_profile("time")
    T = r.get_solution_variable_profile("temperature")
    assert np.all(np.isfinite(T)) and np.all(T > 900.0)
    for sp in ("H2", "O2", "H2O"):
        assert np.all(np.isfinite(r.get_solution_variable_profile(sp)))
    # the run stopped at the end of the first step past T0 + 400 K: the trajectory ends there
    assert t[-1] < 5.0e-4
    assert t[-1] >= tau_ms * 1e-3 * (1 - 1e-12)
    assert np.all(np.diff(t) > 0)
    assert T[-1] >= 1400.0 - 1e-6
    m = r.get_solution_mixture_at_index(len(t) - 1)
    assert abs(m.temperature - T[-1]) < 1e-9
