"""Instruction histogram of reactor_kernel<54, false, false> in an ISA probe (scripts/isa_probe.sh)."""
import collections
import re
import sys

lines = open(sys.argv[1] if len(sys.argv) > 1 else "/tmp/ckmi_probe.s").read().split("\n")
st = [i for i, l in enumerate(lines) if re.match(r"^_ZN12_GLOBAL__N_114reactor_kernelILi54ELb0ELb0E.*:", l)][0]
en = [i for i in range(st, len(lines)) if "s_endpgm" in lines[i]][0]
c = collections.Counter(l.strip().split(" ")[0] for l in lines[st:en] if l.strip() and not l.strip().startswith((".", ";")))
keys = ["v_mov_b32_e32", "ds_write_b128", "ds_read_b128", "v_fmac_f64_e32", "v_fma_f64", "scratch_store_dword", "s_and_saveexec_b64", "v_readfirstlane_b32",
        "scratch_load_dword", "s_waitcnt"]
print(" ".join(f"{k}={c[k]}" for k in keys), "total", sum(c.values()))
