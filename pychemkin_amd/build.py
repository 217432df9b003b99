"""Build libckmi.so for gfx950 with hipcc (in-tree, so the .so travels with the repo)."""
from __future__ import annotations

import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "ckmi.hip")        # kinetics, thermo and reactor kernels + C ABI
LU_SRC = os.path.join(HERE, "csrc", "ckmi_lu.hip")  # batched MFMA LU (large mechanisms)
BIG_SRC = os.path.join(HERE, "csrc", "ckmi_big.hip")  # workgroup-per-reactor integrator (64 <= KK + 1 <= 192)
BIG_HDR = os.path.join(HERE, "csrc", "ckmi_big_matrix.hpp")  # its register-resident Newton matrix forms
KIN_SRC = os.path.join(HERE, "csrc", "ckmi_kin.cpp")  # KIN-compatible host shims (include/ckmi_kin.h)
JIT_SRC = os.path.join(HERE, "csrc", "ckmi_jit.cpp")  # mechanism-specialised ROP kernel generator (hipRTC)
PARSE_SRC = os.path.join(HERE, "csrc", "ckmi_parse.cpp")  # native Chemkin-II interpreter (KINPreProcess)
TRAN_SRC = os.path.join(HERE, "csrc", "ckmi_transport.hip")  # viscosity fits + species / mixture viscosity
DEPS = [os.path.join(HERE, "csrc", f) for f in ("ckmi_device.hpp", "ckmi_reactor.hpp", "ckmi_image.hpp",
                                                "ckmi_run.hpp", "ckmi_internal.hpp")] + [
    os.path.join(HERE, "..", "include", "ckmi.h"), os.path.join(HERE, "..", "include", "ckmi_kin.h")]
OUT = os.path.join(HERE, "_lib", "libckmi.so")
OBJ_DIR = os.path.join(HERE, "_lib", "obj")
ARCH = "gfx950"  # MI355X only
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")

# MachineLICM / MachineSink are off: in the persistent reactor kernel they hoist FP64
# constants and addresses out of the integrator loop, keep them live across the RHS and then
# spill them to scratch (284 -> 16 B/lane of scratch, +29 % reactors/s measured A/B on MI355X).
FLAGS = ["-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-mcode-object-version=5",
         f"--offload-arch={ARCH}", "-mllvm", "-disable-machine-licm", "-mllvm", "-disable-machine-sink",
         # the Gauss-Jordan factorisation is a fully unrolled 54 x 54 loop nest (a[] must stay in VGPRs)
         "-mllvm", "-pragma-unroll-threshold=2000000"]
LU_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-mcode-object-version=5", f"--offload-arch={ARCH}"]
# the workgroup-per-reactor kernel: same LICM / sink reasoning as FLAGS (its NB x NB register matrix
# must stay in the unified VGPR + AGPR file, no scratch)
BIG_FLAGS = ["-O3", "-std=c++17", "-fPIC", "-munsafe-fp-atomics", "-mcode-object-version=5", f"--offload-arch={ARCH}",
             "-mllvm", "-disable-machine-licm", "-mllvm", "-disable-machine-sink",
             "-mllvm", "-pragma-unroll-threshold=2000000",
             # the blocked Gauss-Jordan's MFMA accumulators are the register-resident matrix itself:
             # VGPR-form MFMA (1249 -> 24 spilled VGPRs at NB = 11)
             "-mllvm", "-amdgpu-mfma-vgpr-form"]
KIN_FLAGS = ["-O2", "-std=c++17", "-fPIC", "-Wall", f"--offload-arch={ARCH}"]  # host code only


def _stale(target: str, sources) -> bool:
    if not os.path.exists(target):
        return True
    t = os.path.getmtime(target)
    return any(os.path.getmtime(p) > t for p in sources)


def needs_build() -> bool:
    return _stale(OUT, [SRC, LU_SRC, BIG_SRC, KIN_SRC, JIT_SRC, PARSE_SRC, TRAN_SRC] + DEPS)


PROF_OUT = os.path.join(HERE, "_lib", "libckmi_prof.so")  # diagnostic phase-timer build


def _compile(src: str, obj: str, flags, verbose: bool) -> None:
    cmd = [HIPCC] + list(flags) + ["-c", "-o", obj, src]
    if verbose:
        print(" ".join(cmd), file=sys.stderr)
    subprocess.run(cmd, check=True)


def build(force: bool = False, verbose: bool = False, prof: bool = False, out: str = None, extra=()) -> str:
    """Build libckmi.so (or the phase-timer build, or an A/B variant at `out` with `extra` flags).

    Separately compiled translation units (the reactor kernel alone takes ~2 min) linked into one
    shared library: ckmi.hip, ckmi_lu.hip, ckmi_big.hip and the host-only ckmi_kin.cpp,
    ckmi_parse.cpp and ckmi_jit.cpp (linked with libhiprtc)."""
    default = out is None and not prof and not extra
    out = out or (PROF_OUT if prof else OUT)
    if not force and default and not needs_build():
        return OUT
    os.makedirs(OBJ_DIR, exist_ok=True)
    jobs = []  # (src, obj, flags): independent translation units, compiled concurrently
    lu_obj = os.path.join(OBJ_DIR, "ckmi_lu.o")
    if force or _stale(lu_obj, [LU_SRC, DEPS[-1]]):
        jobs.append((LU_SRC, lu_obj, LU_FLAGS))
    # variant flags naming the workgroup kernel (-DCKMI_BIG_...) also build a variant of ckmi_big.hip
    big_extra = [f for f in extra if "CKMI_BIG" in f]
    big_tag = "prof" if prof else ("main" if not big_extra else "v_" + os.path.splitext(os.path.basename(out))[0])
    big_obj = os.path.join(OBJ_DIR, "ckmi_big.o" if default else f"ckmi_big_{big_tag}.o")
    if force or big_extra or _stale(big_obj, [BIG_SRC, BIG_HDR] + DEPS):
        jobs.append((BIG_SRC, big_obj, BIG_FLAGS + (["-DCKMI_PHASE_TIMERS"] if prof else []) + big_extra))
    kin_obj = os.path.join(OBJ_DIR, "ckmi_kin.o")
    if force or _stale(kin_obj, [KIN_SRC] + DEPS):
        jobs.append((KIN_SRC, kin_obj, KIN_FLAGS))
    jit_obj = os.path.join(OBJ_DIR, "ckmi_jit.o")
    if force or _stale(jit_obj, [JIT_SRC] + DEPS):
        jobs.append((JIT_SRC, jit_obj, KIN_FLAGS))
    parse_obj = os.path.join(OBJ_DIR, "ckmi_parse.o")
    if force or _stale(parse_obj, [PARSE_SRC] + DEPS):
        jobs.append((PARSE_SRC, parse_obj, KIN_FLAGS))
    tran_obj = os.path.join(OBJ_DIR, "ckmi_transport.o")
    if force or _stale(tran_obj, [TRAN_SRC] + DEPS):
        jobs.append((TRAN_SRC, tran_obj, LU_FLAGS))
    # a variant that only names the workgroup kernel shares the default build's ckmi.hip object
    main_extra = [f for f in extra if "CKMI_BIG" not in f]
    # (a phase-timer build never shares the production object, and vice versa)
    tag = "prof" if prof else ("main" if (default or not main_extra)
                               else os.path.splitext(os.path.basename(out))[0])
    main_obj = os.path.join(OBJ_DIR, f"ckmi_{tag}.o")
    if force or (tag not in ("main", "prof")) or (prof and main_extra) or _stale(main_obj, [SRC] + DEPS):
        jobs.append((SRC, main_obj, FLAGS + (["-DCKMI_PHASE_TIMERS"] if prof else []) + list(main_extra)))
    with ThreadPoolExecutor(max_workers=max(1, min(len(jobs), os.cpu_count() or 1))) as pool:
        for f in [pool.submit(_compile, s, o, fl, verbose) for s, o, fl in jobs]:
            f.result()
    cmd = [HIPCC, "-shared", "-fPIC", f"--offload-arch={ARCH}", "-o", out, main_obj, lu_obj, big_obj, kin_obj, jit_obj,
           parse_obj, tran_obj,
           "-L/opt/rocm/lib", "-lhiprtc", "-Wl,-rpath,/opt/rocm/lib"]
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
