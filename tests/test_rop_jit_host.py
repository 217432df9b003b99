"""Host side of the mechanism-specialised ROP kernel (ckmi_jit.cpp): source generation and a
hipRTC compile for gfx950 -- no GPU needed (the GPU parity tests are test_gpu_rop_jit.py)."""
import pytest

from pychemkin_amd import _native


def test_generated_source_covers_every_reaction_and_species(tables, mech):
    src = _native.rop_jit_source(tables)
    assert 'extern "C" __global__' in src and f"ckjit_rop_k{mech.KK}_i{mech.II}(" in src
    for i in range(mech.II):
        assert f"// reaction {i + 1}\n" in src
    for k in range(mech.KK):
        assert f"// species {k}\n" in src
        assert f"wd[{k} * ns + s]" in src  # every wdot row is stored exactly once
    assert src.count("wd[") == mech.KK


def test_generated_source_compiles_with_hiprtc(tables):
    assert _native.rop_jit_compile(tables) > 10000


EXT = {
    "plog": ("gri30_plog_chem.inp", "grimech30_thermo.dat", ("const double* t0 = prm + ", "lnP")),
    "cheb": ("gri30_cheb_chem.inp", "grimech30_thermo.dat", ("const double Tr = fma(", "t13")),
    "ford": ("gri30_ford_chem.inp", "grimech30_thermo.dat", ("jcpow_lt1(", "lnPRT")),
    "ext161": ("gri30_tracer161_ext_chem.inp", "gri30_tracer161_thermo.dat", ("const double* t0 = prm + ", "jcpow_")),
}


@pytest.mark.parametrize("name", sorted(EXT))
def test_every_reaction_form_has_a_specialised_kernel(name):
    """PLOG, Chebyshev, Landau-Teller, chemically activated, FORD / RORD / fractional and wide
    reactions are generated (round 2 declined such mechanisms) and the source compiles for gfx950."""
    import os

    from conftest import ROOT

    from pychemkin_amd.mechanism import Mechanism

    chem, therm, marks = EXT[name]
    m = Mechanism.from_files(os.path.join(ROOT, "data", chem), os.path.join(ROOT, "data", therm))
    t = m.to_tables()
    src = _native.rop_jit_source(t)
    for i in range(m.II):
        assert f"// reaction {i + 1}\n" in src
    assert src.count("wd[") == m.KK
    for mark in marks:
        assert mark in src, mark
    assert _native.rop_jit_compile(t) > 10000
