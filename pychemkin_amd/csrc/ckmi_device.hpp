// ckmi_device.hpp -- device-side building blocks for gfx950 (CDNA4, wave64).
//
// Wave utilities (DPP reductions, broadcasts) and the global-memory mechanism tables (MechDev,
// used by the thread-per-state species-thermo kernel and for the reaction-order map; the rate
// kernels read the LDS image of ckmi_image.hpp).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ckmi {

constexpr int WAVE = 64;
constexpr int SLOTS = 4;
constexpr double BOLTZMANN = 1.3806504e-16;
constexpr double AVOGADRO = 6.02214179e23;
constexpr double RU = BOLTZMANN * AVOGADRO;  // erg/mol-K (reference constants.py:37)
constexpr double PATM = 1.01325e6;           // dyn/cm2  (reference constants.py:28)
constexpr double LN_PATM_RU = -4.407419774071825;  // ln(PATM / RU): ln(PATM / (RU T)) = LN_PATM_RU - ln T

// Device-resident mechanism tables.  Reactions are re-ordered by type (elementary first,
// then third-body, then falloff) so that a 64-lane strip is type-uniform; `orig` maps a
// device slot back to the reference reaction index.  All per-reaction arrays have IIpad
// entries (pad slots carry nr = np = 0 and produce nothing).
struct MechDev {
  int KK, II, IIpad, G;
  const double* wt;     // [KK]
  const double* rwt;    // [KK] 1/W
  const double* th;     // [17][KK] tlow, tmid, thigh, low a1..a7, high a1..a7 (coefficient-major)
  const int* flags;     // [IIpad] type | rev<<2 | has_rev<<3 | ftype<<4
  const int* nrp;       // [IIpad] nr | np<<8
  const int4* rsp;      // [IIpad]
  const int4* psp;      // [IIpad]
  const double* rnu;    // [SLOTS][IIpad]
  const double* pnu;    // [SLOTS][IIpad]
  const double* lnA;    // [IIpad]
  const double* beta;
  const double* Ea;     // E/R
  const double* lnA0;   // low-pressure limit
  const double* beta0;
  const double* Ea0;
  const double* fp;     // [5][IIpad] TROE / SRI
  const double* rlnA;   // explicit REV
  const double* rbeta;
  const double* rEa;
  const double* dnu;    // [IIpad] sum(nu'') - sum(nu')
  const double* ordf;   // [IIpad] sum(nu')
  const double* ordr;   // [IIpad] sum(nu'')
  const int* tb;        // [IIpad] >=0 third-body group, <= -2 collider species -(tb+2), -1 none
  const int* orig;      // [IIpad] original reaction index, -1 for pad
  const int* gptr;      // [G+1]
  const int* gsp;
  const double* geff;   // efficiency - 1
};

// ------------------------------------------------------------------ wave utilities
__device__ __forceinline__ double uni(double v) {
  // make a value provably wave-uniform (lives in SGPRs afterwards)
  const int lo = __builtin_amdgcn_readfirstlane(__double2loint(v));
  const int hi = __builtin_amdgcn_readfirstlane(__double2hiint(v));
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }

__device__ __forceinline__ double bcast(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ int bcast(int v, int lane) { return __builtin_amdgcn_readlane(v, lane); }

// Cross-lane reductions on the DPP path (quad_perm / row_half_mirror / row_mirror inside each
// 16-lane row, then four readlanes across rows): no LDS round trips, unlike ds_bpermute-based
// __shfl_xor.  Every lane of a row computes the same commutative pairings, so the result is
// identical in all lanes and deterministic.
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
constexpr int DPP_QUAD_1032 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int DPP_QUAD_2301 = 0x4E;  // quad_perm [2,3,0,1]
constexpr int DPP_ROW_HALF_MIRROR = 0x141;
constexpr int DPP_ROW_MIRROR = 0x140;

// Across the four rows: the gfx950 row swaps (v_permlane16_swap pairs rows 0-1 and 2-3,
// v_permlane32_swap the two halves) hand every lane its partner row's value, so each lane forms
// (s0 + s1) + (s2 + s3) itself -- the association of the readlane form, bitwise, without the 8
// readlanes and their SGPR round trip.  A/B form (CKMI_REDUCE_SWAP): bitwise the same results, no faster
// (c3 244.7 vs 243.1 ms, c5 438.7 vs 439.5 ms on the A/B samples, profiles/r05_ab_reduce_swap_*.log).
template <bool HALVES>
__device__ __forceinline__ void row_swap(double v, double& own, double& other) {
  const uint32_t lo = (uint32_t)__double2loint(v), hi = (uint32_t)__double2hiint(v);
  const auto l = HALVES ? __builtin_amdgcn_permlane32_swap(lo, lo, false, false)
                        : __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h = HALVES ? __builtin_amdgcn_permlane32_swap(hi, hi, false, false)
                        : __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  own = __hiloint2double((int)h[0], (int)l[0]);  // {own, partner} in a row-dependent order:
  other = __hiloint2double((int)h[1], (int)l[1]);  // only commutative combinations of the two
}
__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_mov<DPP_QUAD_1032>(v);
  v += dpp_mov<DPP_QUAD_2301>(v);
  v += dpp_mov<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_mov<DPP_ROW_MIRROR>(v);
#ifndef CKMI_REDUCE_SWAP
  return uni((bcast(v, 0) + bcast(v, 16)) + (bcast(v, 32) + bcast(v, 48)));
#else
  double a, b;
  row_swap<false>(v, a, b);
  v = a + b;
  row_swap<true>(v, a, b);
  return uni(a + b);
#endif
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_mov<DPP_QUAD_1032>(v));
  v = fmax(v, dpp_mov<DPP_QUAD_2301>(v));
  v = fmax(v, dpp_mov<DPP_ROW_HALF_MIRROR>(v));
  v = fmax(v, dpp_mov<DPP_ROW_MIRROR>(v));
#ifndef CKMI_REDUCE_SWAP
  return uni(fmax(fmax(bcast(v, 0), bcast(v, 16)), fmax(bcast(v, 32), bcast(v, 48))));
#else
  double a, b;
  row_swap<false>(v, a, b);
  v = fmax(a, b);
  row_swap<true>(v, a, b);
  return uni(fmax(a, b));
#endif
}

// max of a u32 over the wave (DPP inside rows, readlanes across them); the pivot search
// compares |a| as fp32 bit patterns: 1 VALU op per stage instead of 3 for an FP64 fmax
__device__ __forceinline__ uint32_t wave_max_u32(uint32_t v) {
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_QUAD_1032, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_QUAD_2301, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_ROW_HALF_MIRROR, 0xf, 0xf, false));
  v = max(v, (uint32_t)__builtin_amdgcn_mov_dpp((int)v, DPP_ROW_MIRROR, 0xf, 0xf, false));
  const uint32_t a = __builtin_amdgcn_readlane(v, 0), b = __builtin_amdgcn_readlane(v, 16);
  const uint32_t c = __builtin_amdgcn_readlane(v, 32), d = __builtin_amdgcn_readlane(v, 48);
  return max(max(a, b), max(c, d));
}

// 1 / x from the hardware reciprocal and two Newton steps (no IEEE division sequence)
__device__ __forceinline__ double rcp_nr(double x) {
  double r = __builtin_amdgcn_rcp(x);
  double e = fma(-x, r, 1.0);
  r = fma(r, e, r);
  e = fma(-x, r, 1.0);
  return fma(r, e, r);
}

// ------------------------------------------------------------------ thermo (NASA-7)
struct SpThermo {
  double cpR, hRT, sR;
};
__device__ __forceinline__ SpThermo nasa7(const MechDev& M, int k, double T, double lnT) {
  const int KK = M.KK;
  const double tmid = M.th[1 * KK + k];
  const int base = (T > tmid) ? 10 : 3;
  const double a0 = M.th[(base + 0) * KK + k], a1 = M.th[(base + 1) * KK + k], a2 = M.th[(base + 2) * KK + k];
  const double a3 = M.th[(base + 3) * KK + k], a4 = M.th[(base + 4) * KK + k], a5 = M.th[(base + 5) * KK + k];
  const double a6 = M.th[(base + 6) * KK + k];
  const double T2 = T * T, T3 = T2 * T, T4 = T3 * T;
  SpThermo r;
  r.cpR = a0 + a1 * T + a2 * T2 + a3 * T3 + a4 * T4;
  r.hRT = a0 + a1 * T / 2 + a2 * T2 / 3 + a3 * T3 / 4 + a4 * T4 / 5 + a5 / T;
  r.sR = a0 * lnT + a1 * T + a2 * T2 / 2 + a3 * T3 / 3 + a4 * T4 / 4 + a6;
  return r;
}

}  // namespace ckmi
