"""Build libckmi.so for gfx950 with hipcc (in-tree, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "ckmi.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("ckmi_device.hpp", "ckmi_reactor.hpp", "ckmi_image.hpp")] + [
    os.path.join(HERE, "..", "include", "ckmi.h")]
OUT = os.path.join(HERE, "_lib", "libckmi.so")
ARCH = "gfx950"  # MI355X only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# MachineLICM / MachineSink are off: in the persistent reactor kernel they hoist FP64
# constants and addresses out of the integrator loop, keep them live across the RHS and then
# spill them to scratch (284 -> 16 B/lane of scratch, +29 % reactors/s measured A/B on MI355X).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics", "-mcode-object-version=5",
         f"--offload-arch={ARCH}", "-mllvm", "-disable-machine-licm", "-mllvm", "-disable-machine-sink",
         # the Gauss-Jordan factorisation is a fully unrolled 54 x 54 loop nest (a[] must stay in VGPRs)
         "-mllvm", "-pragma-unroll-threshold=2000000"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in [SRC] + DEPS)


PROF_OUT = os.path.join(HERE, "_lib", "libckmi_prof.so")  # diagnostic phase-timer build


def build(force: bool = False, verbose: bool = False, prof: bool = False, out: str = None, extra=()) -> str:
    """Build libckmi.so (or the phase-timer build, or an A/B variant at `out` with `extra` flags)."""
    default = out is None and not prof and not extra
    out = out or (PROF_OUT if prof else OUT)
    if not force and default and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [HIPCC] + FLAGS + (["-DCKMI_PHASE_TIMERS"] if prof else []) + list(extra) + ["-o", out, SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    # python build.py [--force] [--prof] [--out PATH] [-- extra hipcc flags...]
    argv = sys.argv[1:]
    extra = argv[argv.index("--") + 1:] if "--" in argv else []
    argv = argv[:argv.index("--")] if "--" in argv else argv
    out = argv[argv.index("--out") + 1] if "--out" in argv else None
    print(build(force="--force" in argv, verbose=True, prof="--prof" in argv, out=out, extra=extra))
