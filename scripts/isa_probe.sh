#!/bin/bash
# Register / scratch figures of the configs[2] reactor kernel (reactor_kernel<54, false, false>) from a
# one-variant device compile (-DCKMI_PROBE_C3; CPU only, no GPU).  Extra arguments are passed to hipcc
# (e.g. -DSOME_VARIANT).   Usage: scripts/isa_probe.sh [hipcc flags...]
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${ISA_OUT:-/tmp/ckmi_probe.s}
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC -munsafe-fp-atomics -mcode-object-version=5 --offload-arch=gfx950 \
  -mllvm -disable-machine-licm -mllvm -disable-machine-sink -mllvm -pragma-unroll-threshold=2000000 \
  --offload-device-only -S -DCKMI_PROBE_C3 "$@" -o "$OUT" "$ROOT/pychemkin_amd/csrc/ckmi.hip"
K=_ZN12_GLOBAL__N_114reactor_kernelILi54ELb0ELb0EEEvN4ckmi9MechImageEPKNS1_6DevCfgEiiPiPdNS1_9ReactorIOE
for f in num_vgpr numbered_sgpr private_seg_size; do  # (num_vgpr may print nothing when it is an expression)
  grep -m1 "\.set $K\.$f," "$OUT" | sed "s/.*\.$f, /$f /"
done
