// ckmi_internal.hpp -- host-side internals shared by the translation units of libckmi.so.
#pragma once
#include <hip/hip_runtime.h>

#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "ckmi_device.hpp"
#include "ckmi_image.hpp"

struct ckmi_mech {
  int device;
  int KK, II, IIpad, G;
  ckmi::MechDev d;
  ckmi::MechImage img;  // compact LDS image (device copy in img.blob)
  std::vector<void*> allocs;
  // host copies of the forward Arrhenius (original order) for get/set
  std::vector<double> lnA_orig, b_orig, E_orig;
  std::vector<int> rtype_orig;
  bool has_plog = false;
  std::vector<int> slot_of;  // original reaction -> device slot
};

namespace ckmi {
struct DevCfg;
struct ReactorIO;
// record the message for ckmi_last_error() and return code
int set_error(int code, const std::string& msg);
// one workgroup per reactor: 64 <= KK + 1 <= 192 (ckmi_big.hip)
int launch_big_reactors(const ckmi_mech* m, int n, const DevCfg& dc, const ReactorIO& io, hipStream_t stream);
}  // namespace ckmi
