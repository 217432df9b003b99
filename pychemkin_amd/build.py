"""Build libckmi.so for gfx950 with hipcc (in-tree, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "ckmi.hip")
DEPS = [os.path.join(HERE, "csrc", f) for f in ("ckmi_device.hpp", "ckmi_reactor.hpp")] + [
    os.path.join(HERE, "..", "include", "ckmi.h")]
OUT = os.path.join(HERE, "_lib", "libckmi.so")
ARCH = "gfx950"  # MI355X only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

FLAGS = ["-O3", "-std=c++17", "-fPIC", "-shared", "-munsafe-fp-atomics", "-mcode-object-version=5",
         f"--offload-arch={ARCH}"]


def needs_build() -> bool:
    if not os.path.exists(OUT):
        return True
    t = os.path.getmtime(OUT)
    return any(os.path.getmtime(p) > t for p in [SRC] + DEPS)


PROF_OUT = os.path.join(HERE, "_lib", "libckmi_prof.so")  # diagnostic phase-timer build


def build(force: bool = False, verbose: bool = False, prof: bool = False) -> str:
    out = PROF_OUT if prof else OUT
    if not force and not prof and not needs_build():
        return OUT
    os.makedirs(os.path.dirname(out), exist_ok=True)
    cmd = [HIPCC] + FLAGS + (["-DCKMI_PHASE_TIMERS"] if prof else []) + ["-o", out, SRC]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)
    return out


if __name__ == "__main__":
    print(build(force="--force" in sys.argv, verbose=True, prof="--prof" in sys.argv))
