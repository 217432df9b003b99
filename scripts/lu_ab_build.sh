#!/bin/bash
# Standalone LU builds for scripts/lu_ab.py (the default form).
# Variants of ckmi_lu.hip under test are compiled the same way, from a copy of the file.
set -e
cd "$(dirname "$0")/.."
mkdir -p pychemkin_amd/_lib/ab
F="-O3 -std=c++17 -fPIC -shared -mcode-object-version=5 --offload-arch=gfx950 -mllvm -pragma-unroll-threshold=2000000"
/opt/rocm/bin/hipcc $F -o pychemkin_amd/_lib/ab/lu_base.so pychemkin_amd/csrc/ckmi_lu.hip &
wait
