// ckmi_internal.hpp -- host-side internals shared by the translation units of libckmi.so.
#pragma once
#include <hip/hip_runtime.h>

#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "ckmi_device.hpp"
#include "ckmi_image.hpp"

namespace ckmi {
// mechanism-specialised ROP kernel (ckmi_jit.cpp): source generated at ckmi_mech_create, compiled
// with hipRTC at the first call that selects it
struct JitRop {
  std::string src, why;
  std::vector<int> lnA_off;  // original reaction -> offset of its ln A in the parameter block
  double* prm = nullptr;     // device parameter block
  std::atomic<int> state{0};  // 0 not compiled yet, 1 ready, -1 unsupported / compile failed (why, under mu)
  hipModule_t mod = nullptr;
  hipFunction_t fn = nullptr;
  std::mutex mu;
};
// A reaction the unit-coefficient slots cannot express: a non-integral (or < 1) stoichiometric
// coefficient, a FORD / RORD order that differs from the coefficient, or more than 4 molecules
// on a side.  Evaluated by the extended kernel variants (ckmi_image.hpp eval_gen_img).
// Slot counts within 0..CKMI_SLOTS and species indices within 0..KK-1 for every reaction, checked
// before any table walk (a descriptor from the C ABI is untrusted); nullptr when valid.
inline const char* check_slots(const ckmi_mech_desc* d) {
  if (!d->nr || !d->np || !d->rsp || !d->psp || !d->rnu || !d->pnu) return "null reaction tables";
  for (int i = 0; i < d->II; ++i) {
    if (d->nr[i] < 0 || d->nr[i] > CKMI_SLOTS || d->np[i] < 0 || d->np[i] > CKMI_SLOTS)
      return "more than 4 species on one side of a reaction (nr / np outside 0..4)";
    for (int u = 0; u < d->nr[i]; ++u)
      if (d->rsp[CKMI_SLOTS * i + u] < 0 || d->rsp[CKMI_SLOTS * i + u] >= d->KK) return "reactant species index out of range";
    for (int u = 0; u < d->np[i]; ++u)
      if (d->psp[CKMI_SLOTS * i + u] < 0 || d->psp[CKMI_SLOTS * i + u] >= d->KK) return "product species index out of range";
  }
  return nullptr;
}
inline bool rxn_general(const ckmi_mech_desc* d, int i) {
  int mr = 0, mp = 0;
  for (int u = 0; u < d->nr[i]; ++u) {
    const double nu = d->rnu[CKMI_SLOTS * i + u];
    if (nu != (double)(int)nu || nu < 1.0) return true;
    if (d->ford && d->ford[CKMI_SLOTS * i + u] != nu) return true;
    mr += (int)nu;
  }
  for (int u = 0; u < d->np[i]; ++u) {
    const double nu = d->pnu[CKMI_SLOTS * i + u];
    if (nu != (double)(int)nu || nu < 1.0) return true;
    if (d->rord && d->rord[CKMI_SLOTS * i + u] != nu) return true;
    mp += (int)nu;
  }
  return mr > 4 || mp > 4 || d->nr[i] > 4 || d->np[i] > 4;
}
bool jit_rop_generate(const ckmi_mech_desc* d, std::string& src, std::vector<double>& prm, std::vector<int>& lnA_off,
                      std::string& why);
int jit_rop_compile(const std::string& src, std::vector<char>& code, std::string& log);
}  // namespace ckmi

struct ckmi_mech {
  int device;
  int KK, II, IIpad, G;
  ckmi::MechDev d;
  ckmi::MechImage img;  // compact LDS image (device copy in img.blob)
  std::vector<void*> allocs;
  // host copies of the forward Arrhenius (original order) for get/set
  std::vector<double> lnA_orig, b_orig, E_orig;
  std::vector<int> rtype_orig;
  bool has_plog = false;     // PLOG / chemically activated / general reactions: extended kernel variants
  bool has_general = false;  // FORD / RORD / non-integral coefficients (rxn_general)
  std::vector<int> slot_of;  // original reaction -> device slot
  double tguard_lo = 0.0, tguard_hi = 1e300;  // runaway guard: min_k T_low,k / 2, max_k T_high,k
  int npe = 0;  // elements of the corrector's element projection (image element table), 0 = none
  ckmi::JitRop* jit = nullptr;
};

namespace ckmi {
struct DevCfg;
struct ReactorIO;
// record the message for ckmi_last_error() and return code
int set_error(int code, const std::string& msg);
// one workgroup per reactor: 64 <= KK + 1 <= 192 (ckmi_big.hip)
int launch_big_reactors(const ckmi_mech* m, int n, const DevCfg& dc, const ReactorIO& io, hipStream_t stream);
}  // namespace ckmi
