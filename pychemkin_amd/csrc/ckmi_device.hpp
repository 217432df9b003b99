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

__device__ __forceinline__ double wave_sum(double v) {
  v += dpp_mov<DPP_QUAD_1032>(v);
  v += dpp_mov<DPP_QUAD_2301>(v);
  v += dpp_mov<DPP_ROW_HALF_MIRROR>(v);
  v += dpp_mov<DPP_ROW_MIRROR>(v);
  return uni((bcast(v, 0) + bcast(v, 16)) + (bcast(v, 32) + bcast(v, 48)));
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_mov<DPP_QUAD_1032>(v));
  v = fmax(v, dpp_mov<DPP_QUAD_2301>(v));
  v = fmax(v, dpp_mov<DPP_ROW_HALF_MIRROR>(v));
  v = fmax(v, dpp_mov<DPP_ROW_MIRROR>(v));
  return uni(fmax(fmax(bcast(v, 0), bcast(v, 16)), fmax(bcast(v, 32), bcast(v, 48))));
}

// ------------------------------------------------------------------ multi-value wave sums
// NV values per lane summed over the wave in one pass: a reduce-scatter over the six lane bits, each
// stage halving the registers (the lane's bit picks which one of a pair it keeps; its partner gets the
// other), then plain all-reduce stages once one register is left.  Stages: bit 5 by v_permlane32_swap,
// bit 4 by v_permlane16_swap (each pairs two registers in one instruction per dword: no selects), bits
// 3 / 2 / 1 / 0 by DPP row_mirror / row_half_mirror / quad_perm (partners 15 - i, 7 - i, i ^ 2, i ^ 1 of
// the 16-lane row).  8 values: 4 + 2 + 1 pair stages + 3 all-reduce stages (~34 VALU issues) instead of 8
// wave_sums (~180).  The sum of value j ends in the lanes whose bits 5, 4, 3, .. are the binary digits
// 0, 1, 2, .. of j (wave_sum_lane); the association is fixed, so results are deterministic and the same
// in every wave.
__device__ __forceinline__ void swap_rows(double& a, double& b, bool halves) {
  const uint32_t al = (uint32_t)__double2loint(a), ah = (uint32_t)__double2hiint(a);
  const uint32_t bl = (uint32_t)__double2loint(b), bh = (uint32_t)__double2hiint(b);
  const auto l = halves ? __builtin_amdgcn_permlane32_swap(al, bl, false, false)
                        : __builtin_amdgcn_permlane16_swap(al, bl, false, false);
  const auto h = halves ? __builtin_amdgcn_permlane32_swap(ah, bh, false, false)
                        : __builtin_amdgcn_permlane16_swap(ah, bh, false, false);
  a = __hiloint2double((int)h[0], (int)l[0]);
  b = __hiloint2double((int)h[1], (int)l[1]);
}
template <int S>
__device__ __forceinline__ double dpp_partner(double v) {  // stage S = 2..5: the partner across lane bit 5 - S
  if constexpr (S == 2) return dpp_mov<DPP_ROW_MIRROR>(v);
  else if constexpr (S == 3) return dpp_mov<DPP_ROW_HALF_MIRROR>(v);
  else if constexpr (S == 4) return dpp_mov<DPP_QUAD_2301>(v);
  else return dpp_mov<DPP_QUAD_1032>(v);
}
template <int S, int R, int NV>
__device__ __forceinline__ void wave_sum_stages(double (&v)[NV], int lane) {
  if constexpr (S < 6) {
    if constexpr (R > 1) {
#pragma unroll
      for (int j = 0; j < R / 2; ++j) {
        double a = v[2 * j], b = v[2 * j + 1];
        if constexpr (S < 2) {
          swap_rows(a, b, S == 0);  // lanes with bit 5 - S clear: a = (own, partner) of v[2j], else of v[2j+1]
          v[j] = a + b;
        } else {
          const bool hi = (lane >> (5 - S)) & 1;
          const double send = hi ? a : b, keep = hi ? b : a;
          v[j] = keep + dpp_partner<S>(send);
        }
      }
      wave_sum_stages<S + 1, R / 2>(v, lane);
    } else {
      if constexpr (S < 2) {
        double a = v[0], b = v[0];
        swap_rows(a, b, S == 0);
        v[0] = a + b;
      } else {
        v[0] += dpp_partner<S>(v[0]);
      }
      wave_sum_stages<S + 1, 1>(v, lane);
    }
  }
}
// the lane holding the sum of value j (any lane with these upper bits holds it)
__device__ __forceinline__ constexpr int wave_sum_lane(int j) {
  return ((j & 1) << 5) | ((j & 2) << 3) | ((j & 4) << 1) | ((j & 8) >> 1) | ((j & 16) >> 3) | ((j & 32) >> 5);
}
// the value index a lane holds after wave_sum_multi<NV> (inverse of wave_sum_lane on the top log2 NV bits)
template <int NV>
__device__ __forceinline__ int wave_sum_index(int lane) {
  int j = 0;
#pragma unroll
  for (int s = 0; (1 << s) < NV; ++s) j |= ((lane >> (5 - s)) & 1) << s;
  return j;
}
// v[j] <- sum over the wave of v[j], in every lane (wave-uniform); NV a power of two <= 64
template <int NV>
__device__ __forceinline__ void wave_sum_multi(double (&v)[NV], int lane) {
  wave_sum_stages<0, NV>(v, lane);
  const double x = v[0];
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = bcast(x, wave_sum_lane(j));
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
