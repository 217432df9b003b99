"""ctypes binding of libckmi.so (include/ckmi.h) -- the product's native path.

Mirrors the reference's FFI layer (``chemkin_wrapper.py:244,271-272,300-867``): one
``ctypes.CDLL`` loaded at import, prototypes declared once, ``int`` status returns.  Device
buffers are torch tensors on the ROCm device; torch is imported first so that libckmi binds
to the same HIP runtime instance (both carry SONAME ``libamdhip64.so.7``).

There is no CPU fallback: if the library is missing or no GPU is present, the calls raise.
"""
from __future__ import annotations

import ctypes as ct
import os
from typing import Dict, Optional

import numpy as np
import torch  # noqa: F401  (must be loaded before libckmi.so)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CKMI_LIB selects another in-tree build of the same ABI (the phase-timer diagnostic build,
# _lib/libckmi_prof.so, used by scripts/phase_profile.py); it is never a CPU path.
LIB_PATH = os.environ.get("CKMI_LIB") or os.path.join(_HERE, "_lib", "libckmi.so")

ABI_VERSION = 3  # CKMI_ABI_VERSION (include/ckmi.h): the layouts of MechDesc / ReactorCfg below
NSTAT = 8
STAT_NAMES = ("nst", "nfe", "nje", "nlu", "ncf", "nef", "status", "nni")
RUN_STATUS = {0: "ok", 1: "max_steps", 2: "error_test_failures", 3: "convergence_failures", 4: "runaway",
              5: "choked"}


class NativeError(RuntimeError):
    pass


_P = ct.c_void_p


class MechDesc(ct.Structure):
    _fields_ = [("KK", ct.c_int32), ("II", ct.c_int32)] + [
        (n, _P) for n in ("wt", "thermo", "rtype", "rev", "nr", "np", "rsp", "psp", "rnu", "pnu", "arr", "low",
                          "revp", "has_rev", "ftype", "fpar", "tbsp", "eff_ptr", "eff_sp", "eff_val",
                          "plog_ptr", "plog_par", "ford", "rord")
    ] + [("MM", ct.c_int32), ("ncf", _P)]


# the pointer fields of MechDesc (MM is a count, ncf optional: tables without element counts leave the
# element projection off)
_DESC_PTRS = [n for n, t in MechDesc._fields_[2:] if t is _P and n != "ncf"]


def fill_desc(d: "MechDesc", tables: Dict[str, np.ndarray], keep: Dict[str, np.ndarray]) -> None:
    d.KK, d.II = int(tables["KK"]), int(tables["II"])
    for name in _DESC_PTRS:
        setattr(d, name, keep[name].ctypes.data)
    if "ncf" in keep and "MM" in tables:
        d.MM, d.ncf = int(tables["MM"]), keep["ncf"].ctypes.data
    else:
        d.MM, d.ncf = 0, None


class ReactorCfg(ct.Structure):
    _fields_ = [
        ("energy", ct.c_int32), ("t_end", ct.c_double), ("atol", ct.c_double), ("rtol", ct.c_double),
        ("h0", ct.c_double), ("hmax", ct.c_double), ("nneg", ct.c_int32), ("ign_mode", ct.c_int32),
        ("ign_val", ct.c_double), ("ign_species", ct.c_int32), ("ign_stop", ct.c_int32), ("max_steps", ct.c_int32),
        ("nprof", ct.c_int32), ("prof_t", ct.c_double * 64), ("prof_v", ct.c_double * 64),
        ("prof_kind", ct.c_int32), ("gfac", ct.c_double), ("qloss", ct.c_double), ("htc", ct.c_double),
        ("areaq", ct.c_double), ("tamb", ct.c_double), ("asteps", ct.c_int32), ("avar", ct.c_int32),
        ("avalue", ct.c_double), ("nprof2", ct.c_int32), ("prof2_kind", ct.c_int32), ("prof2_t", ct.c_double * 64),
        ("prof2_v", ct.c_double * 64), ("nprof3", ct.c_int32), ("prof3_t", ct.c_double * 64),
        ("prof3_v", ct.c_double * 64), ("eng", ct.c_double * 20), ("tran", _P), ("no_elem_proj", ct.c_int32),
    ]


class ReactorExt(ct.Structure):
    _fields_ = [("afac_rxn", _P), ("afac", _P), ("max_adap", ct.c_int32), ("t_adap", _P), ("y_adap", _P),
                ("n_adap", _P), ("t_stop", _P)]


_lib: Optional[ct.CDLL] = None

# every symbol include/ckmi.h declares, with its prototype
PROTOTYPES = {
    "ckmi_last_error": (ct.c_char_p, []),
    "ckmi_version": (ct.c_int, []),
    "ckmi_mech_create": (ct.c_int, [ct.POINTER(MechDesc), ct.POINTER(_P)]),
    "ckmi_mech_destroy": (ct.c_int, [_P]),
    "ckmi_mech_sizes": (ct.c_int, [_P, ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32)]),
    "ckmi_get_arrhenius": (ct.c_int, [_P, _P, _P, _P]),
    "ckmi_set_afactor": (ct.c_int, [_P, ct.c_int32, ct.c_double]),
    "ckmi_species_thermo": (ct.c_int, [_P, ct.c_int32, _P, _P, _P, _P, _P]),
    "ckmi_rop_thermo": (ct.c_int, [_P, ct.c_int32, _P, _P, _P, _P, _P, _P, _P]),
    "ckmi_reaction_rates": (ct.c_int, [_P, ct.c_int32, _P, _P, _P, _P, _P, _P]),
    "ckmi_reactor_run": (ct.c_int, [_P, ct.POINTER(ReactorCfg), ct.c_int32, _P, _P, _P, _P, _P, _P, _P, _P, _P, _P,
                                     _P, ct.c_int32, _P, _P, _P]),
    "ckmi_reactor_run_ex": (ct.c_int, [_P, ct.POINTER(ReactorCfg), ct.c_int32, _P, _P, _P, _P, _P,
                                        ct.POINTER(ReactorExt), _P, _P, _P, _P, _P, _P, ct.c_int32, _P, _P, _P]),
    "ckmi_engine_heat_rates": (ct.c_int, [_P, ct.POINTER(ReactorCfg), ct.c_double, ct.c_double, _P, ct.c_int32, _P, _P,
                                          _P, _P, _P]),
    "ckmi_set_reactor_path": (ct.c_int, [ct.c_int32]),
    "ckmi_big_max_image_bytes": (ct.c_int, [ct.c_int32, ct.c_int32, ct.c_int32, ct.c_int32]),
    "ckmi_set_rop_path": (ct.c_int, [ct.c_int32]),
    "ckmi_rop_jit_state": (ct.c_int, [_P, ct.POINTER(ct.c_int32)]),
    "ckmi_rop_jit_source": (ct.c_int, [ct.POINTER(MechDesc), ct.c_char_p, ct.c_int64, ct.POINTER(ct.c_int64)]),
    "ckmi_rop_jit_compile": (ct.c_int, [ct.POINTER(MechDesc), ct.POINTER(ct.c_int64)]),
    "ckmi_lu_factor_batched": (ct.c_int, [ct.c_int32, ct.c_int32, _P, _P, _P, _P]),
    "ckmi_lu_solve_batched": (ct.c_int, [ct.c_int32, ct.c_int32, _P, _P, _P, _P]),
    "ckmi_lu_last_error": (ct.c_char_p, []),
    "ckmi_parse_mechanism": (ct.c_int, [ct.c_char_p, ct.c_char_p, ct.POINTER(_P)]),
    "ckmi_parse_files": (ct.c_int, [ct.c_char_p, ct.c_char_p, ct.POINTER(_P)]),
    "ckmi_parse_last_error": (ct.c_char_p, []),
    "ckmi_parsed_free": (None, [_P]),
    "ckmi_parsed_sizes": (ct.c_int, [_P, ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32), ct.POINTER(ct.c_int32)]),
    "ckmi_parsed_desc": (ct.c_int, [_P, ct.POINTER(MechDesc)]),
    "ckmi_parsed_symbols": (ct.c_int, [_P, _P, _P, _P, _P]),
    "ckmi_parsed_equation": (ct.c_int, [_P, ct.c_int32, ct.c_char_p, ct.c_int32, ct.POINTER(ct.c_int32)]),
    "ckmi_transport_fit": (ct.c_int, [ct.c_int32, _P, _P, ct.c_double, ct.c_double, _P]),
    "ckmi_conductivity_fit": (ct.c_int, [ct.c_int32, _P, _P, _P, ct.c_double, ct.c_double, _P]),
    "ckmi_transport_create": (ct.c_int, [_P, _P, ct.POINTER(_P)]),
    "ckmi_transport_destroy": (ct.c_int, [_P]),
    "ckmi_transport_fits": (ct.c_int, [_P, _P]),
    "ckmi_species_viscosity": (ct.c_int, [_P, ct.c_int32, _P, _P, _P]),
    "ckmi_mixture_viscosity": (ct.c_int, [_P, ct.c_int32, _P, _P, _P, _P]),
    "ckmi_transport_set_conductivity": (ct.c_int, [_P, _P]),
    "ckmi_species_conductivity": (ct.c_int, [_P, ct.c_int32, _P, _P, _P]),
    "ckmi_mixture_conductivity": (ct.c_int, [_P, ct.c_int32, _P, _P, _P, _P]),
}
LU_NMAX = 192


def lib() -> ct.CDLL:
    """Load libckmi.so once (raises if it was not built: no silent fallback)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise NativeError(f"libckmi.so not found at {LIB_PATH}; run __graft_entry__.build()")
        L = ct.CDLL(LIB_PATH)
        for name, (res, args) in PROTOTYPES.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        if L.ckmi_version() != ABI_VERSION:
            raise NativeError(f"{LIB_PATH} has ABI version {L.ckmi_version()}, this binding needs {ABI_VERSION}; "
                              "rebuild with __graft_entry__.build()")
        _lib = L
    return _lib


def _check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ckmi_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (code {rc}): {msg}")


SLOTS = 8  # CKMI_SLOTS (include/ckmi.h): distinct species per reaction side of the flat tables

# ckmi_mech_desc fields -> (dtype, shape given KK, II, npl)
_DESC_LAYOUT = {
    "wt": (np.float64, lambda K, I, n: (K,)), "thermo": (np.float64, lambda K, I, n: (K, 17)),
    "rtype": (np.int32, lambda K, I, n: (I,)), "rev": (np.int32, lambda K, I, n: (I,)),
    "nr": (np.int32, lambda K, I, n: (I,)), "np": (np.int32, lambda K, I, n: (I,)),
    "rsp": (np.int32, lambda K, I, n: (I, SLOTS)), "psp": (np.int32, lambda K, I, n: (I, SLOTS)),
    "rnu": (np.float64, lambda K, I, n: (I, SLOTS)), "pnu": (np.float64, lambda K, I, n: (I, SLOTS)),
    "arr": (np.float64, lambda K, I, n: (I, 3)), "low": (np.float64, lambda K, I, n: (I, 3)),
    "revp": (np.float64, lambda K, I, n: (I, 3)), "has_rev": (np.int32, lambda K, I, n: (I,)),
    "ftype": (np.int32, lambda K, I, n: (I,)), "fpar": (np.float64, lambda K, I, n: (I, 5)),
    "tbsp": (np.int32, lambda K, I, n: (I,)), "eff_ptr": (np.int32, lambda K, I, n: (I + 1,)),
    "plog_ptr": (np.int32, lambda K, I, n: (I + 1,)),
    "ford": (np.float64, lambda K, I, n: (I, SLOTS)), "rord": (np.float64, lambda K, I, n: (I, SLOTS)),
}


def parse_mechanism(chem_text: str, therm_text: str = ""):
    """Run libckmi's native Chemkin interpreter (the parse half of KINPreProcess; host only, no GPU).

    Returns (tables, species, elements, awt, ncf, equations) with ``tables`` in the layout of
    ``Mechanism.to_tables()``; raises NativeError with the interpreter's message on a bad file."""
    L = lib()
    h = _P()
    rc = L.ckmi_parse_mechanism(chem_text.encode(), (therm_text or "").encode(), ct.byref(h))
    if rc != 0:
        raise NativeError(f"ckmi_parse_mechanism failed (code {rc}): "
                          f"{L.ckmi_parse_last_error().decode(errors='replace')}")
    try:
        MM, KK, II = ct.c_int32(), ct.c_int32(), ct.c_int32()
        L.ckmi_parsed_sizes(h, ct.byref(MM), ct.byref(KK), ct.byref(II))
        MM, KK, II = MM.value, KK.value, II.value
        d = MechDesc()
        L.ckmi_parsed_desc(h, ct.byref(d))
        ne = int(np.ctypeslib.as_array(ct.cast(d.eff_ptr, ct.POINTER(ct.c_int32)), (II + 1,))[-1])
        npl = int(np.ctypeslib.as_array(ct.cast(d.plog_ptr, ct.POINTER(ct.c_int32)), (II + 1,))[-1])
        t = {"KK": np.int32(KK), "II": np.int32(II)}
        for name, (dt, shp) in _DESC_LAYOUT.items():
            cty = ct.c_double if dt == np.float64 else ct.c_int32
            t[name] = np.ctypeslib.as_array(ct.cast(getattr(d, name), ct.POINTER(cty)), shp(KK, II, npl)).copy()
        t["eff_sp"] = np.ctypeslib.as_array(ct.cast(d.eff_sp, ct.POINTER(ct.c_int32)), (max(ne, 1),))[:ne].copy()
        t["eff_val"] = np.ctypeslib.as_array(ct.cast(d.eff_val, ct.POINTER(ct.c_double)), (max(ne, 1),))[:ne].copy()
        t["plog_par"] = np.ctypeslib.as_array(ct.cast(d.plog_par, ct.POINTER(ct.c_double)),
                                              (max(npl, 1), 4)).copy()
        t["MM"] = np.int32(d.MM)
        t["ncf"] = np.ctypeslib.as_array(ct.cast(d.ncf, ct.POINTER(ct.c_int32)), (MM, KK)).copy()
        sp = ct.create_string_buffer(16 * KK + 1)
        el = ct.create_string_buffer(16 * MM + 1)
        awt = np.zeros(MM)
        ncf = np.zeros((MM, KK), np.int32)
        L.ckmi_parsed_symbols(h, ct.addressof(sp), ct.addressof(el), awt.ctypes.data, ncf.ctypes.data)
        species = [sp.raw[16 * k:16 * k + 16].rstrip(b"\0").decode() for k in range(KK)]
        elements = [el.raw[16 * m:16 * m + 16].rstrip(b"\0").decode() for m in range(MM)]
        eqs = []
        buf = ct.create_string_buffer(4096)
        n = ct.c_int32()
        for i in range(II):
            L.ckmi_parsed_equation(h, i, buf, 4096, ct.byref(n))
            eqs.append(buf.value.decode())
        return t, species, elements, awt, ncf, eqs
    finally:
        L.ckmi_parsed_free(h)


def _ptr(t) -> Optional[int]:
    if t is None:
        return None
    if isinstance(t, np.ndarray):
        return t.ctypes.data
    return t.data_ptr()


def _stream_ptr(device) -> int:
    return torch.cuda.current_stream(device).cuda_stream


IGN_MODES = {None: 0, "none": 0, "T_inflection": 1, "TIFP": 1, "T_rise": 2, "DTIGN": 2, "T_ignition": 3,
             "TLIM": 3, "Species_peak": 4, "KLIM": 4}


def make_cfg(energy: int = 1, t_end: float = 1.0, atol: float = 1e-12, rtol: float = 1e-6, h0: float = 0.0,
             hmax: float = 0.0, nneg: bool = False, ign_mode=None, ign_val: float = 0.0, ign_species: int = 0,
             ign_stop: bool = False, max_steps: int = 0, profile=None, prof_kind: int = 0, gfac: float = 1.0,
             qloss: float = 0.0, htc: float = 0.0, areaq: float = 0.0, tamb: float = 300.0,
             asteps: int = 0, avar: int = -1, avalue: float = 0.0, profile2=None, prof2_kind: int = 0,
             profile3=None, engine=None, tran=None, elem_proj: bool = True) -> ReactorCfg:
    """Typed form of the reactor keywords (see include/ckmi.h ckmi_reactor_cfg).

    profile: (x, v) VPRO/PPRO (prof_kind 0) or TPRO (prof_kind 1); profile2: (x, v) QPRO
    (prof2_kind 1) or AEXT (prof2_kind 2); profile3: (x, v) AEXT beside a QPRO profile2; engine: the
    CKMI_ENG_* parameter block of problem 4 (<= 20 values); tran: device tensor [KK][8] of viscosity and
    conductivity fits (the engine's ICHX heat transfer), kept alive by the returned struct; elem_proj=False
    turns off the element projection of the corrector (diagnostics; include/ckmi.h no_elem_proj)."""
    c = ReactorCfg()
    c.no_elem_proj = 0 if elem_proj else 1
    if engine is not None:
        e = np.asarray(engine, np.float64)
        if e.size > 20:
            raise ValueError("engine block has at most 20 values")
        for i, v in enumerate(e):
            c.eng[i] = float(v)
    if tran is not None:
        if not isinstance(tran, torch.Tensor) or tran.dtype != torch.float64 or not tran.is_cuda:
            raise ValueError("tran must be a float64 device tensor [KK][8]")
        c.tran = tran.data_ptr()
        c._tran_keep = tran
    c.avar, c.avalue = int(avar), float(avalue)
    c.nprof2, c.prof2_kind = 0, int(prof2_kind)
    if profile2 is not None:
        x2, v2 = np.asarray(profile2[0], np.float64), np.asarray(profile2[1], np.float64)
        if len(x2) != len(v2) or len(x2) > 64 or len(x2) == 0:
            raise ValueError("profile2 must have matching lengths in [1, 64]")
        c.nprof2 = len(x2)
        for i in range(len(x2)):
            c.prof2_t[i] = x2[i]
            c.prof2_v[i] = v2[i]
    c.nprof3 = 0
    if profile3 is not None:
        x3, v3 = np.asarray(profile3[0], np.float64), np.asarray(profile3[1], np.float64)
        if len(x3) != len(v3) or len(x3) > 64 or len(x3) == 0:
            raise ValueError("profile3 must have matching lengths in [1, 64]")
        c.nprof3 = len(x3)
        for i in range(len(x3)):
            c.prof3_t[i] = x3[i]
            c.prof3_v[i] = v3[i]
    c.prof_kind, c.gfac, c.qloss, c.htc, c.areaq, c.tamb = int(prof_kind), float(gfac), float(qloss), float(htc), \
        float(areaq), float(tamb)
    c.asteps = int(asteps)
    c.energy, c.t_end, c.atol, c.rtol = int(energy), float(t_end), float(atol), float(rtol)
    c.h0, c.hmax, c.nneg = float(h0), float(hmax), int(bool(nneg))
    c.ign_mode = IGN_MODES[ign_mode] if not isinstance(ign_mode, int) else int(ign_mode)
    c.ign_val, c.ign_species, c.ign_stop, c.max_steps = float(ign_val), int(ign_species), int(bool(ign_stop)), int(max_steps)
    c.nprof = 0
    if profile is not None:
        x, v = np.asarray(profile[0], np.float64), np.asarray(profile[1], np.float64)
        if len(x) != len(v) or len(x) > 64:
            raise ValueError("profile must have matching lengths <= 64")
        c.nprof = len(x)
        for i in range(len(x)):
            c.prof_t[i] = x[i]
            c.prof_v[i] = v[i]
    return c


def mech_desc(tables: Dict[str, np.ndarray]):
    """ckmi_mech_desc view of flat mechanism tables; returns (desc, arrays kept alive)."""
    keep = {k: np.ascontiguousarray(v) for k, v in tables.items() if isinstance(v, np.ndarray) and v.ndim > 0}
    d = MechDesc()
    fill_desc(d, tables, keep)
    return d, keep


def rop_jit_source(tables: Dict[str, np.ndarray]) -> str:
    """Source of the mechanism-specialised ROP kernel (host only, no GPU)."""
    d, keep = mech_desc(tables)
    n = ct.c_int64(0)
    _check(lib().ckmi_rop_jit_source(ct.byref(d), None, 0, ct.byref(n)), "ckmi_rop_jit_source")
    buf = ct.create_string_buffer(n.value + 1)
    _check(lib().ckmi_rop_jit_source(ct.byref(d), buf, n.value + 1, ct.byref(n)), "ckmi_rop_jit_source")
    del keep
    return buf.value.decode()


def rop_jit_compile(tables: Dict[str, np.ndarray]) -> int:
    """Compile the specialised ROP kernel with hipRTC (no GPU); returns the code object size."""
    d, keep = mech_desc(tables)
    n = ct.c_int64(0)
    _check(lib().ckmi_rop_jit_compile(ct.byref(d), ct.byref(n)), "ckmi_rop_jit_compile")
    del keep
    return int(n.value)


def set_rop_path(path: int) -> None:
    """0 automatic, 1 generic reaction-per-lane kernel, 2 mechanism-specialised kernel."""
    _check(lib().ckmi_set_rop_path(int(path)), "ckmi_set_rop_path")


class DeviceMechanism:
    """Mechanism tables resident in HBM of one GPU (wraps a ckmi_mech handle)."""

    def __init__(self, tables: Dict[str, np.ndarray], device=None):
        if not torch.cuda.is_available():
            raise NativeError("no ROCm GPU visible: the ckmi device path requires an MI355X")
        self.device = torch.device("cuda", torch.cuda.current_device() if device is None else torch.device(device).index or 0)
        self.KK = int(tables["KK"])
        self.II = int(tables["II"])
        keep = {k: np.ascontiguousarray(v) for k, v in tables.items() if isinstance(v, np.ndarray) and v.ndim > 0}
        d = MechDesc()
        fill_desc(d, tables, keep)
        h = _P()
        with torch.cuda.device(self.device):
            _check(lib().ckmi_mech_create(ct.byref(d), ct.byref(h)), "ckmi_mech_create")
        self._h = h
        del keep

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ckmi_mech_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    def rop_jit_state(self) -> int:
        """Specialised ROP kernel of this mechanism: 0 not compiled yet, 1 ready, -1 unavailable."""
        st = ct.c_int32(0)
        _check(lib().ckmi_rop_jit_state(self._h, ct.byref(st)), "ckmi_rop_jit_state")
        return int(st.value)

    # -------------------------------------------------------------- parameters
    def arrhenius(self):
        A, b, E = (np.zeros(self.II) for _ in range(3))
        _check(lib().ckmi_get_arrhenius(self._h, A.ctypes.data, b.ctypes.data, E.ctypes.data), "ckmi_get_arrhenius")
        return A, b, E

    def set_afactor(self, irxn: int, A: float) -> None:
        with torch.cuda.device(self.device):
            _check(lib().ckmi_set_afactor(self._h, int(irxn), float(A)), "ckmi_set_afactor")

    # -------------------------------------------------------------- helpers
    def _dev(self, x, dtype=torch.float64):
        if isinstance(x, torch.Tensor):
            return x.to(device=self.device, dtype=dtype).contiguous()
        return torch.as_tensor(np.ascontiguousarray(x), dtype=dtype, device=self.device)

    # -------------------------------------------------------------- kernels
    def species_thermo(self, T):
        T = self._dev(T).reshape(-1)
        n = T.numel()
        cp, h, s = (torch.empty((self.KK, n), dtype=torch.float64, device=self.device) for _ in range(3))
        with torch.cuda.device(self.device):
            _check(lib().ckmi_species_thermo(self._h, n, _ptr(T), _ptr(cp), _ptr(h), _ptr(s),
                                             _stream_ptr(self.device)), "ckmi_species_thermo")
        return cp, h, s

    def rop_thermo(self, T, P, Y_soa, wdot=None, cp=None, h=None):
        """T[n], P[n], Y[KK][n] -> wdot[KK][n], cp[n], h[n] (all device tensors)."""
        T = self._dev(T).reshape(-1)
        P = self._dev(P).reshape(-1)
        Y = self._dev(Y_soa)
        n = T.numel()
        if Y.shape != (self.KK, n):
            raise ValueError(f"Y must be [KK={self.KK}][n={n}], got {tuple(Y.shape)}")
        if wdot is None:
            wdot = torch.empty((self.KK, n), dtype=torch.float64, device=self.device)
        if cp is None:
            cp = torch.empty(n, dtype=torch.float64, device=self.device)
        if h is None:
            h = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):  # the specialised kernel's module lives on this device
            _check(lib().ckmi_rop_thermo(self._h, n, _ptr(T), _ptr(P), _ptr(Y), _ptr(wdot), _ptr(cp), _ptr(h),
                                         _stream_ptr(self.device)), "ckmi_rop_thermo")
        return wdot, cp, h

    def reaction_rates(self, T, P, Y_soa):
        T = self._dev(T).reshape(-1)
        P = self._dev(P).reshape(-1)
        Y = self._dev(Y_soa)
        n = T.numel()
        qf = torch.empty((self.II, n), dtype=torch.float64, device=self.device)
        qr = torch.empty((self.II, n), dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            _check(lib().ckmi_reaction_rates(self._h, n, _ptr(T), _ptr(P), _ptr(Y), _ptr(qf), _ptr(qr),
                                             _stream_ptr(self.device)), "ckmi_reaction_rates")
        return qf, qr

    def reactor_run(self, cfg: ReactorCfg, problem, T0, P0, V0, Y0, t_save=None, out=None, afac_rxn=None, afac=None,
                    max_adap: int = 0):
        """Integrate n independent reactors. Y0 is [n][KK]. Returns a dict of device tensors.

        afac_rxn / afac: per-reactor A-factor perturbation (reaction index, multiplier), the
        batched form of the reference's sensitivity loop (sensitivity.py:141-160).
        max_adap > 0 with cfg.asteps > 0: adaptive solution points (t_adap, y_adap, n_adap)."""
        if not isinstance(problem, torch.Tensor):
            pv = np.asarray(problem)
            if pv.size and not np.all((pv >= 1) & (pv <= 4)):
                raise NativeError("problem must be 1 (CONP), 2 (CONV), 3 (plug flow) or 4 (engine) for every reactor")
        T0 = self._dev(T0).reshape(-1)
        n = T0.numel()
        P0 = self._dev(P0).reshape(-1)
        V0 = self._dev(V0).reshape(-1)
        Y0 = self._dev(Y0).reshape(n, self.KK)
        prob = self._dev(problem, torch.int32).reshape(-1)
        if not (P0.numel() == V0.numel() == prob.numel() == n):
            raise ValueError("T0, P0, V0, problem must all have n entries")
        o = out or {}
        dev = self.device
        f64 = dict(dtype=torch.float64, device=dev)
        tau = o.get("tau", torch.empty(n, **f64))
        Tend = o.get("T", torch.empty(n, **f64))
        Pend = o.get("P", torch.empty(n, **f64))
        Vend = o.get("V", torch.empty(n, **f64))
        Yend = o.get("Y", torch.empty((n, self.KK), **f64))
        stats = o.get("stats", torch.empty((n, NSTAT), dtype=torch.int32, device=dev))
        t_stop = o.get("t_stop", torch.empty(n, **f64))
        nsave = 0
        ts = ys = None
        if t_save is not None:
            ts = self._dev(t_save).reshape(-1)
            nsave = ts.numel()
            ys = torch.empty((n, nsave, self.KK + 1), **f64)
        ext = ReactorExt()
        ext.t_stop = _ptr(t_stop)
        keep = []
        if afac_rxn is not None:
            ar = self._dev(afac_rxn, torch.int32).reshape(-1)
            af = self._dev(afac).reshape(-1)
            if ar.numel() != n or af.numel() != n:
                raise ValueError("afac_rxn and afac must have n entries")
            if bool((af <= 0).any()):
                raise NativeError("A-factor multipliers must be > 0")
            ext.afac_rxn, ext.afac = _ptr(ar), _ptr(af)
            keep += [ar, af]
        adap = None
        if max_adap > 0:
            adap = dict(t_adap=torch.zeros((n, max_adap), **f64), y_adap=torch.zeros((n, max_adap, self.KK + 1), **f64),
                        n_adap=torch.zeros(n, dtype=torch.int32, device=dev))
            ext.max_adap = int(max_adap)
            ext.t_adap, ext.y_adap, ext.n_adap = _ptr(adap["t_adap"]), _ptr(adap["y_adap"]), _ptr(adap["n_adap"])
        _check(lib().ckmi_reactor_run_ex(self._h, ct.byref(cfg), n, _ptr(prob), _ptr(T0), _ptr(P0), _ptr(V0),
                                         _ptr(Y0), ct.byref(ext), _ptr(tau), _ptr(Tend), _ptr(Pend), _ptr(Vend),
                                         _ptr(Yend), _ptr(stats), nsave, _ptr(ts), _ptr(ys), _stream_ptr(dev)),
               "ckmi_reactor_run_ex")
        res = dict(tau=tau, T=Tend, P=Pend, V=Vend, Y=Yend, stats=stats, t_stop=t_stop)
        if adap is not None:
            res.update(adap)
        if keep:
            # the per-reactor A-factor inputs stay referenced by the result: the launch is
            # asynchronous on this stream, and the caching allocator may only reuse their memory
            # for work ordered after it (no host synchronisation needed)
            res["_inputs"] = keep
        if ys is not None:
            res["t_save"] = ts
            res["y_save"] = ys
        return res

    def engine_heat_rates(self, cfg: ReactorCfg, T0: float, P0: float, Y0, t, y):
        """Apparent heat-release and wall heat-loss rates [erg/s] of an engine run (problem 4) on its
        saved states t[n], y[n][KK+1], from the integrator's own right-hand side
        (ckmi_engine_heat_rates; the output side of KINAll0D_GetEngineHeatRelease, engine.py:953-988)."""
        Y0 = self._dev(Y0).reshape(-1)
        t = self._dev(t).reshape(-1)
        n = t.numel()
        y = self._dev(y).reshape(n, self.KK + 1)
        if Y0.numel() != self.KK:
            raise ValueError(f"Y0 must have KK = {self.KK} entries")
        ahrr = torch.empty(n, dtype=torch.float64, device=self.device)
        qloss = torch.empty(n, dtype=torch.float64, device=self.device)
        with torch.cuda.device(self.device):
            _check(lib().ckmi_engine_heat_rates(self._h, ct.byref(cfg), float(T0), float(P0), _ptr(Y0), n, _ptr(t),
                                                _ptr(y), _ptr(ahrr), _ptr(qloss), _stream_ptr(self.device)),
                   "ckmi_engine_heat_rates")
        return ahrr, qloss


def transport_fit(wt: np.ndarray, params: np.ndarray, tlow: float, thigh: float) -> np.ndarray:
    """Viscosity fits [KK][4] (ln eta_k as a cubic in ln T) from TRANLIB parameters [KK][6]; host only."""
    wt = np.ascontiguousarray(wt, dtype=np.float64)
    params = np.ascontiguousarray(params, dtype=np.float64)
    KK = wt.shape[0]
    if params.shape != (KK, 6):
        raise NativeError(f"transport parameters must be [{KK}][6], got {params.shape}")
    fits = np.zeros((KK, 4))
    _check(lib().ckmi_transport_fit(KK, wt.ctypes.data, params.ctypes.data, float(tlow), float(thigh),
                                    fits.ctypes.data), "ckmi_transport_fit")
    return fits


def conductivity_fit(wt: np.ndarray, params: np.ndarray, thermo: np.ndarray, tlow: float, thigh: float) -> np.ndarray:
    """Thermal conductivity fits [KK][4] (ln lambda_k as a cubic in ln T) from TRANLIB parameters [KK][6]
    and the NASA-7 table [KK][17]; host only."""
    wt = np.ascontiguousarray(wt, dtype=np.float64)
    params = np.ascontiguousarray(params, dtype=np.float64)
    thermo = np.ascontiguousarray(thermo, dtype=np.float64)
    KK = wt.shape[0]
    if params.shape != (KK, 6) or thermo.shape != (KK, 17):
        raise NativeError(f"need params [{KK}][6] and thermo [{KK}][17], got {params.shape}, {thermo.shape}")
    fits = np.zeros((KK, 4))
    _check(lib().ckmi_conductivity_fit(KK, wt.ctypes.data, params.ctypes.data, thermo.ctypes.data, float(tlow),
                                       float(thigh), fits.ctypes.data), "ckmi_conductivity_fit")
    return fits


class DeviceTransport:
    """Viscosity (and optionally conductivity) fits and Wilke tables of one DeviceMechanism, on its GPU
    (wraps ckmi_transport)."""

    def __init__(self, dm: "DeviceMechanism", fits: np.ndarray, cond_fits: Optional[np.ndarray] = None):
        self.dm = dm
        self.KK = dm.KK
        fits = np.ascontiguousarray(fits, dtype=np.float64)
        if fits.shape != (self.KK, 4):
            raise NativeError(f"viscosity fits must be [{self.KK}][4], got {fits.shape}")
        h = _P()
        with torch.cuda.device(dm.device):
            _check(lib().ckmi_transport_create(dm.handle, fits.ctypes.data, ct.byref(h)), "ckmi_transport_create")
        self._h = h
        self.has_conductivity = False
        if cond_fits is not None:
            cf = np.ascontiguousarray(cond_fits, dtype=np.float64)
            if cf.shape != (self.KK, 4):
                raise NativeError(f"conductivity fits must be [{self.KK}][4], got {cf.shape}")
            with torch.cuda.device(dm.device):
                _check(lib().ckmi_transport_set_conductivity(self._h, cf.ctypes.data), "ckmi_transport_set_conductivity")
            self.has_conductivity = True

    def close(self):
        if getattr(self, "_h", None) is not None and self._h.value:
            lib().ckmi_transport_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def fits(self) -> np.ndarray:
        out = np.zeros((self.KK, 4))
        _check(lib().ckmi_transport_fits(self._h, out.ctypes.data), "ckmi_transport_fits")
        return out

    def species_viscosity(self, T) -> torch.Tensor:
        """T[n] -> eta[KK][n] [g/(cm s)] (device tensor)."""
        T = self.dm._dev(T).reshape(-1)
        n = T.numel()
        out = torch.empty((self.KK, n), dtype=torch.float64, device=self.dm.device)
        with torch.cuda.device(self.dm.device):
            _check(lib().ckmi_species_viscosity(self._h, n, _ptr(T), _ptr(out), _stream_ptr(self.dm.device)),
                   "ckmi_species_viscosity")
        return out

    def mixture_viscosity(self, T, Y_soa) -> torch.Tensor:
        """T[n], Y[KK][n] mass fractions -> eta[n] [g/(cm s)] (Wilke; device tensor)."""
        T = self.dm._dev(T).reshape(-1)
        n = T.numel()
        Y = self.dm._dev(Y_soa).reshape(self.KK, n)
        out = torch.empty(n, dtype=torch.float64, device=self.dm.device)
        with torch.cuda.device(self.dm.device):
            _check(lib().ckmi_mixture_viscosity(self._h, n, _ptr(T), _ptr(Y), _ptr(out), _stream_ptr(self.dm.device)),
                   "ckmi_mixture_viscosity")
        return out

    def species_conductivity(self, T) -> torch.Tensor:
        """T[n] -> lambda[KK][n] [erg/(cm s K)] (device tensor; KINGetConductivity x n)."""
        T = self.dm._dev(T).reshape(-1)
        n = T.numel()
        out = torch.empty((self.KK, n), dtype=torch.float64, device=self.dm.device)
        with torch.cuda.device(self.dm.device):
            _check(lib().ckmi_species_conductivity(self._h, n, _ptr(T), _ptr(out), _stream_ptr(self.dm.device)),
                   "ckmi_species_conductivity")
        return out

    def mixture_conductivity(self, T, Y_soa) -> torch.Tensor:
        """T[n], Y[KK][n] mass fractions -> lambda[n] [erg/(cm s K)] (mixture-averaged; device tensor)."""
        T = self.dm._dev(T).reshape(-1)
        n = T.numel()
        Y = self.dm._dev(Y_soa).reshape(self.KK, n)
        out = torch.empty(n, dtype=torch.float64, device=self.dm.device)
        with torch.cuda.device(self.dm.device):
            _check(lib().ckmi_mixture_conductivity(self._h, n, _ptr(T), _ptr(Y), _ptr(out),
                                                   _stream_ptr(self.dm.device)), "ckmi_mixture_conductivity")
        return out


def set_reactor_path(path: int) -> None:
    """0: automatic (wave per reactor for KK + 1 <= 64 -- Newton inverse stored in FP32 unless
    rtol < 1e-9 -- workgroup per reactor above); 1: the workgroup-per-reactor kernel for every
    mechanism (testing both integrators on one mechanism); 2 / 3: the wave kernel with the FP64 /
    FP32-stored Newton inverse whatever the tolerances."""
    _check(lib().ckmi_set_reactor_path(int(path)), "ckmi_set_reactor_path")


# ------------------------------------------------------------------ batched dense LU (n <= 192)
def _lu_check(rc: int, what: str) -> None:
    if rc != 0:
        msg = lib().ckmi_lu_last_error().decode(errors="replace")
        raise NativeError(f"{what} failed (code {rc}): {msg}")


def lu_factor_batched(A: torch.Tensor):
    """In-place batched LU with partial pivoting of A[nsys, n, n] (FP64, row-major, on the GPU).

    Returns (A, ipiv[nsys, n] int32 0-based, info[nsys] int32) with LAPACK dgetrf semantics:
    the Newton-matrix factorisation of the reactor integrator for mechanisms with more than 63
    species (trailing updates on FP64 MFMA)."""
    if not isinstance(A, torch.Tensor) or not A.is_cuda:
        raise NativeError("lu_factor_batched needs a device tensor (no CPU path)")
    if A.dtype != torch.float64 or A.dim() != 3 or A.shape[1] != A.shape[2] or not A.is_contiguous():
        raise ValueError("A must be a contiguous float64 tensor [nsys, n, n]")
    nsys, n = int(A.shape[0]), int(A.shape[1])
    if not 1 <= n <= LU_NMAX:
        raise ValueError(f"n must be in [1, {LU_NMAX}]")
    ipiv = torch.empty((nsys, n), dtype=torch.int32, device=A.device)
    info = torch.empty(nsys, dtype=torch.int32, device=A.device)
    with torch.cuda.device(A.device):
        _lu_check(lib().ckmi_lu_factor_batched(nsys, n, _ptr(A), _ptr(ipiv), _ptr(info), _stream_ptr(A.device)),
                  "ckmi_lu_factor_batched")
    return A, ipiv, info


def lu_solve_batched(LU: torch.Tensor, ipiv: torch.Tensor, B: torch.Tensor) -> torch.Tensor:
    """B[nsys, n] <- A^-1 B in place, from the factors of lu_factor_batched."""
    if not (LU.is_cuda and ipiv.is_cuda and B.is_cuda):
        raise NativeError("lu_solve_batched needs device tensors (no CPU path)")
    nsys, n = int(LU.shape[0]), int(LU.shape[1])
    if tuple(B.shape) != (nsys, n) or B.dtype != torch.float64 or not B.is_contiguous():
        raise ValueError("B must be a contiguous float64 tensor [nsys, n]")
    if tuple(ipiv.shape) != (nsys, n) or ipiv.dtype != torch.int32:
        raise ValueError("ipiv must be int32 [nsys, n]")
    with torch.cuda.device(LU.device):
        _lu_check(lib().ckmi_lu_solve_batched(nsys, n, _ptr(LU), _ptr(ipiv), _ptr(B), _stream_ptr(LU.device)),
                  "ckmi_lu_solve_batched")
    return B
