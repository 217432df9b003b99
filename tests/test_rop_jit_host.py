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


def test_plog_mechanism_has_no_specialised_kernel():
    from conftest import THERM
    from test_plog import PLOG_CHEM

    from pychemkin_amd.mechanism import Mechanism

    pm = Mechanism.from_files(PLOG_CHEM, THERM)
    with pytest.raises(_native.NativeError, match="PLOG"):
        _native.rop_jit_source(pm.to_tables())
