// ckmi_device.hpp -- device-side building blocks for gfx950 (CDNA4, wave64).
//
// Execution model: one 64-lane wavefront owns one reactor (or one state for the ROP
// kernels).  Lane l holds component l of the ODE state y = (T, Y_1..Y_KK); the reaction
// loop is strip-mined over the 64 lanes; species production and the analytic Jacobian are
// assembled in LDS; the Newton iteration matrix is LU-factored row-per-lane in VGPRs.
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

// C^nu for the integral stoichiometric coefficients accepted by ckmi_mech_create
__device__ __forceinline__ double powi_nu(double c, double nu) {
  if (nu == 1.0) return c;
  if (nu == 2.0) return c * c;
  if (nu == 0.0) return 1.0;
  double r = c * c * c;
  for (int k = 3; k < (int)nu; ++k) r *= c;
  return r;
}

__device__ __forceinline__ int slot(const int4& v, int s) {
  return s == 0 ? v.x : (s == 1 ? v.y : (s == 2 ? v.z : v.w));
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

// ------------------------------------------------------------------ one reaction
struct RxnEval {
  double kf, kr, mfac, pf, pr, dlkf, dlkr;
};

// Rate coefficients and concentration products of device reaction slot i at (T, C).
// C, gRT, hRT, Mg live in LDS.  Mirrors oracle/ckoracle.c eval_reaction().
__device__ __forceinline__ RxnEval eval_rxn(const MechDev& M, int i, double T, double lnT, double invT,
                                            double lnPRT, const double* C, const double* gRT, const double* hRT,
                                            const double* Mg, bool need_h) {
  const int fl = M.flags[i];
  const int type = fl & 3;
  const int nrp = M.nrp[i];
  const int nr = nrp & 0xff, np = nrp >> 8;
  const int4 rs = M.rsp[i], ps = M.psp[i];
  const int IIp = M.IIpad;
  const double lnA = M.lnA[i], b = M.beta[i], Ea = M.Ea[i];
  double kf = exp(lnA + b * lnT - Ea * invT);
  const double dlkf = (b + Ea * invT) * invT;
  double mfac = 1.0;
  if (type != 0) {
    const int tb = M.tb[i];
    const double Mc = tb >= 0 ? Mg[tb] : C[-tb - 2];
    if (type == 1) {
      mfac = Mc;
    } else {
      const double k0 = exp(M.lnA0[i] + M.beta0[i] * lnT - M.Ea0[i] * invT);
      const double Pr = k0 * Mc / kf;
      double F = 1.0;
      const int ft = (fl >> 4) & 7;
      if (ft == 2 || ft == 3) {
        const double fa = M.fp[0 * IIp + i], T3s = M.fp[1 * IIp + i], T1s = M.fp[2 * IIp + i];
        double Fcent = (1.0 - fa) * exp(-T / T3s) + fa * exp(-T / T1s);
        if (ft == 3) Fcent += exp(-M.fp[3 * IIp + i] * invT);
        const double lFc = log10(Fcent > 1e-300 ? Fcent : 1e-300);
        const double lPr = log10(Pr > 1e-300 ? Pr : 1e-300);
        const double c = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;
        const double f1 = (lPr + c) / (nn - 0.14 * (lPr + c));
        F = exp10(lFc / (1.0 + f1 * f1));
      } else if (ft == 4) {
        const double lPr = log10(Pr > 1e-300 ? Pr : 1e-300);
        const double X = 1.0 / (1.0 + lPr * lPr);
        F = M.fp[3 * IIp + i] * pow(M.fp[0 * IIp + i] * exp(-M.fp[1 * IIp + i] * invT) + exp(-T / M.fp[2 * IIp + i]), X) *
            pow(T, M.fp[4 * IIp + i]);
      }
      kf = kf * (Pr / (1.0 + Pr)) * F;
    }
  }
  double kr = 0.0, dlkr = 0.0;
  if ((fl >> 2) & 1) {
    if ((fl >> 3) & 1) {
      kr = exp(M.rlnA[i] + M.rbeta[i] * lnT - M.rEa[i] * invT);
      if (type == 2) kr *= kf / exp(lnA + b * lnT - Ea * invT);
      dlkr = (M.rbeta[i] + M.rEa[i] * invT) * invT;
    } else {
      double dG = 0.0, dH = 0.0;
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (s < nr) {
          const int k = slot(rs, s);
          const double nu = M.rnu[s * IIp + i];
          dG -= nu * gRT[k];
          if (need_h) dH -= nu * hRT[k];
        }
      }
#pragma unroll
      for (int s = 0; s < SLOTS; ++s) {
        if (s < np) {
          const int k = slot(ps, s);
          const double nu = M.pnu[s * IIp + i];
          dG += nu * gRT[k];
          if (need_h) dH += nu * hRT[k];
        }
      }
      const double dnu = M.dnu[i];
      kr = kf * exp(dG - dnu * lnPRT);
      dlkr = dlkf - (dH - dnu) * invT;
    }
  }
  double pf = 1.0, pr = 1.0;
#pragma unroll
  for (int s = 0; s < SLOTS; ++s) {
    if (s < nr) pf *= powi_nu(C[slot(rs, s)], M.rnu[s * IIp + i]);
    if (s < np) pr *= powi_nu(C[slot(ps, s)], M.pnu[s * IIp + i]);
  }
  RxnEval e;
  e.kf = kf; e.kr = kr; e.mfac = mfac; e.pf = pf; e.pr = pr; e.dlkf = dlkf; e.dlkr = dlkr;
  return e;
}

}  // namespace ckmi
