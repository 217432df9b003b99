"""Per-process cache of device-resident mechanisms (one ckmi_mech per chemistry set and GPU).

The reference keeps one global, mutable "active chemistry set" inside the closed library
(chemistry.py:46-51,175-219).  Here each Chemistry object owns its parsed tables and, lazily,
one DeviceMechanism per GPU it is used on.
"""
from __future__ import annotations

from typing import Dict, Tuple

_cache: Dict[Tuple[int, int], object] = {}


def device_mechanism(chem, device_index: int = None):
    import torch

    from . import _native

    if device_index is None:
        device_index = torch.cuda.current_device()
    key = (id(chem), int(device_index))
    dm = _cache.get(key)
    if dm is None or dm.version != chem._version:
        with torch.cuda.device(device_index):
            dm = _native.DeviceMechanism(chem._mech.to_tables(), device=torch.device("cuda", device_index))
        dm.version = chem._version
        _cache[key] = dm
    return dm


def drop(chem) -> None:
    for k in [k for k in _tcache if k[0] == id(chem)]:
        _tcache.pop(k).close()
    for k in [k for k in _cache if k[0] == id(chem)]:
        dm = _cache.pop(k)
        dm.close()


_tcache: Dict[Tuple[int, int], object] = {}


def device_transport(chem, device_index: int = None):
    """The chemistry set's viscosity fits + Wilke tables on a GPU (one ckmi_transport per device)."""
    import torch

    from . import _native

    if device_index is None:
        device_index = torch.cuda.current_device()
    dm = device_mechanism(chem, device_index)
    key = (id(chem), int(device_index))
    dt = _tcache.get(key)
    if dt is None or dt.version != chem._version:
        cf = chem.conductivity_fits if chem._tran_params is not None else None
        dt = _native.DeviceTransport(dm, chem._vfits, cf)
        dt.version = chem._version
        _tcache[key] = dt
    return dt
