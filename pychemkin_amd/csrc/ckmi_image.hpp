// ckmi_image.hpp -- compact mechanism image, staged once per workgroup into LDS.
//
// ckmi_mech_create packs every table the rate kernels read into one contiguous byte image
// (~28 KB for GRI-Mech 3.0).  A kernel workgroup copies it from HBM into LDS with 16-byte
// loads once, and all of its waves (one reactor or one state each) then read rate
// parameters, stoichiometry and NASA-7 coefficients at LDS latency instead of L2 latency.
//
// Layout (all per-reaction arrays have IIp entries, per-species arrays KKp; reactions are
// ordered elementary -> third-body -> falloff so a 64-lane strip is type-uniform):
//   th    double [15][KKp]  tmid, low a1..a7, high a1..a7 (coefficient-major: lane = species)
//   wt    double [KKp], rwt double [KKp]
//   lnA, beta, Ea  double [IIp]
//   rsp, psp  u32 [IIp]   four unit-coefficient species slots per side, one byte each: a species
//                         with coefficient 2 occupies two slots; unused slots hold the dummy
//                         species sp_one = KKp - 1 (63 for KK <= 63; KKp = KK + 1 rounded up to
//                         64), whose per-wave C is 1 and g/RT, h/RT are 0, so products and sums
//                         over the four slots need no guards
//   nu        u32 [IIp]   (unused by the device kernels; kept for layout stability)
//   info      u32 [IIp]   type:2 rev:1 hasrev:1 ftype:3 nr:3 np:3 | aux index << 16
//   tb        i32 [IIp]   >= 0 third-body group, <= -2 single collider species -(tb+2), -1 none
//   aux       double [naux][13]  lnA0 b0 E0/R, falloff parameters (TROE: a, 1/T***, 1/T*, T**;
//                                SRI: a, b, 1/c, d, e), REV lnA b E/R, pad (AUXW)
//   gptr i32 [G+1], gsp i32 [ng], geff double [ng]   third-body efficiency lists (eff - 1)
//   geffd double [G][KKp]   the same lists dense (eff - 1, 0 for unlisted species)
//   e2t   double [32]       2^(j/32), the table of fexp (E2T_N)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace ckmi {

// aux record width in doubles: odd, so that the records of consecutive lanes (a falloff strip reads
// ax[0..10] of its own record) start on distinct bank pairs of ds_read_b64 (26-dword stride: conflict-
// free across a 32-lane group; 12 doubles = 24 dwords was 4-way)
constexpr int AUXW = 13;
constexpr int SP_ONE = 63;  // dummy species slot of the reactor kernel's images (KK <= 63)
constexpr int KK_IMAGE_MAX = 255;  // species bytes: the dummy slot KKp - 1 must fit in 8 bits

struct MechImage {
  const uint4* blob;  // device copy of the image
  const int* slot_of; // device: original reaction index -> device slot
  // device: the workgroup kernel's Jacobian columns, CSR over species j: the (device slot i, unit slot sl)
  // pairs whose slot species is j, packed i | sl << 16 (general reactions excluded)
  const int* jcol_ptr;       // [KK + 1]
  const uint32_t* jcol_ent;  // [jcol_ptr[KK]]
  int bytes;          // multiple of 16
  int KK, KKp, II, IIp, G, naux;
  int sp_one;         // dummy species slot (KKp - 1)
  int o_th, o_wt, o_rwt, o_lnA, o_beta, o_Ea, o_rsp, o_psp, o_nu, o_info, o_tb, o_aux, o_gptr, o_gsp, o_geff, o_geffd, o_e2t;
};

// Dynamic LDS of every kernel that stages the image.  Views hold byte OFFSETS into it, not
// pointers, so that every access is re-derived from this __shared__ symbol and compiles to
// ds_* instructions even where a view struct is spilled or passed by reference (a generic
// pointer reloaded from memory would turn every LDS access into a flat_* access).
extern __shared__ __attribute__((aligned(16))) char ck_smem[];
template <typename T>
__device__ __forceinline__ T* lds_at(int off) {
  return reinterpret_cast<T*>(ck_smem + off);
}

struct MechView {
  int KK, KKp, IIp, G;
  int o_th, o_wt, o_rwt, o_lnA, o_beta, o_Ea, o_rsp, o_psp, o_nu, o_info, o_tb, o_aux, o_gptr, o_gsp, o_geff, o_geffd, o_e2t;
  __device__ __forceinline__ const double* th() const { return lds_at<const double>(o_th); }
  __device__ __forceinline__ const double* wt() const { return lds_at<const double>(o_wt); }
  __device__ __forceinline__ const double* rwt() const { return lds_at<const double>(o_rwt); }
  __device__ __forceinline__ const double* lnA() const { return lds_at<const double>(o_lnA); }
  __device__ __forceinline__ const double* beta() const { return lds_at<const double>(o_beta); }
  __device__ __forceinline__ const double* Ea() const { return lds_at<const double>(o_Ea); }
  __device__ __forceinline__ const uint32_t* rsp() const { return lds_at<const uint32_t>(o_rsp); }
  __device__ __forceinline__ const uint32_t* psp() const { return lds_at<const uint32_t>(o_psp); }
  __device__ __forceinline__ const uint32_t* nu() const { return lds_at<const uint32_t>(o_nu); }
  __device__ __forceinline__ const uint32_t* info() const { return lds_at<const uint32_t>(o_info); }
  __device__ __forceinline__ const int* tb() const { return lds_at<const int>(o_tb); }
  __device__ __forceinline__ const double* aux() const { return lds_at<const double>(o_aux); }
  __device__ __forceinline__ const int* gptr() const { return lds_at<const int>(o_gptr); }
  __device__ __forceinline__ const int* gsp() const { return lds_at<const int>(o_gsp); }
  __device__ __forceinline__ const double* geff() const { return lds_at<const double>(o_geff); }
  __device__ __forceinline__ const double* geffd() const { return lds_at<const double>(o_geffd); }
  __device__ __forceinline__ const double* e2t() const { return lds_at<const double>(o_e2t); }
  // the transposed dense third-body table is present (64 x 17 doubles; a 2-double stub otherwise):
  // told by its size, so that the view needs no extra field (every SGPR of it is live in the kernels)
  __device__ __forceinline__ bool mgt() const { return o_e2t - o_geffd > 16; }
};

// view of an image staged at LDS byte offset `base`
__device__ __forceinline__ MechView make_view(int base, const MechImage& I) {
  MechView V;
  V.KK = I.KK;
  V.KKp = I.KKp;
  V.IIp = I.IIp;
  V.G = I.G;
  V.o_th = base + I.o_th;
  V.o_wt = base + I.o_wt;
  V.o_rwt = base + I.o_rwt;
  V.o_lnA = base + I.o_lnA;
  V.o_beta = base + I.o_beta;
  V.o_Ea = base + I.o_Ea;
  V.o_rsp = base + I.o_rsp;
  V.o_psp = base + I.o_psp;
  V.o_nu = base + I.o_nu;
  V.o_info = base + I.o_info;
  V.o_tb = base + I.o_tb;
  V.o_aux = base + I.o_aux;
  V.o_gptr = base + I.o_gptr;
  V.o_gsp = base + I.o_gsp;
  V.o_geff = base + I.o_geff;
  V.o_geffd = base + I.o_geffd;
  V.o_e2t = base + I.o_e2t;
  return V;
}

// All threads of the workgroup copy the image into LDS; ends with a workgroup barrier.
__device__ __forceinline__ void stage_image(int base, const MechImage& I) {
  uint4* dst = lds_at<uint4>(base);
  const int n16 = I.bytes >> 4;
  for (int i = threadIdx.x; i < n16; i += blockDim.x) dst[i] = I.blob[i];
  __syncthreads();
}

// ------------------------------------------------------------------ info / packing helpers
__device__ __forceinline__ int rx_type(uint32_t inf) { return inf & 3; }
__device__ __forceinline__ bool rx_rev(uint32_t inf) { return (inf >> 2) & 1; }
__device__ __forceinline__ bool rx_hasrev(uint32_t inf) { return (inf >> 3) & 1; }
__device__ __forceinline__ int rx_ftype(uint32_t inf) { return (inf >> 4) & 7; }
__device__ __forceinline__ int rx_nr(uint32_t inf) { return (inf >> 7) & 7; }
__device__ __forceinline__ int rx_np(uint32_t inf) { return (inf >> 10) & 7; }
__device__ __forceinline__ int rx_aux(uint32_t inf) { return inf >> 16; }
__device__ __forceinline__ int sp_of(uint32_t packed, int u) { return (packed >> (8 * u)) & 0xff; }
__device__ __forceinline__ int nur_of(uint32_t nu, int u) { return (nu >> (4 * u)) & 0xf; }
__device__ __forceinline__ int nup_of(uint32_t nu, int u) { return (nu >> (16 + 4 * u)) & 0xf; }

// Info bit 15: on a type-3 slot a Chebyshev rate (aux stream NT, NP, 1/Tmin, 1/Tmax, log10 Pmin,
// log10 Pmax, a[t][p]) instead of a PLOG table; on a type-0 slot Landau-Teller terms (aux record:
// B, C at [0], [1]; the RLT B, C of an explicit reverse rate at [3], [4]).  Extended variants only.
constexpr uint32_t RX_ALT = 0x8000u;

// C^nu for a small non-negative integer nu, branch-free for nu <= 3
__device__ __forceinline__ double powi(double c, int nu) {
  double r = nu >= 1 ? c : 1.0;
  r *= nu >= 2 ? c : 1.0;
  r *= nu >= 3 ? c : 1.0;
  if (nu > 3)
    for (int k = 3; k < nu; ++k) r *= c;
  return r;
}

// exp(x) by Tang's table method: x = (32 m + j) ln2/32 + r, |r| <= ln2/64, e^x = 2^m 2^(j/32) e^r
// with a degree-6 polynomial for e^r - 1 (truncation 3e-18 relative at |r| = ln2/64, far below the
// rounding of the result) and the 32-entry table in LDS: 32 doubles are 64 dwords, one per LDS bank,
// so a wave's random-index gathers never conflict (a 64-entry table put entries j and j + 32 on one
// bank pair: ~2-way on most gathers).  ~17 VALU instructions + 1 LDS read instead of ~40 for the
// library exp.  NaN propagates; |x| > 1000 saturates to 0 / inf.
constexpr int E2T_N = 32;
constexpr int E2T_SHIFT = 5;
constexpr double E2T_INV_L = 46.166241308446828;          // 32 / ln 2
constexpr double E2T_L_HI = 0x1.62e42fefa39efp-6;         // (ln 2)_hi / 32
constexpr double E2T_L_LO = 0x1.abc9e3b39803fp-61;        // (ln 2)_lo / 32
__device__ __forceinline__ double fexp(double x, const double* e2t) {
  constexpr double INV_L = E2T_INV_L, L_HI = E2T_L_HI, L_LO = E2T_L_LO;
  x = x < -1000.0 ? -1000.0 : (x > 1000.0 ? 1000.0 : x);
  const double kd = __builtin_rint(x * INV_L);
  const double r = fma(kd, -L_LO, fma(kd, -L_HI, x));
  const int k = (int)kd;
  const double p = fma(r * r,
                       fma(r, fma(r, fma(r, fma(r, 1.0 / 720.0, 1.0 / 120.0), 1.0 / 24.0), 1.0 / 6.0), 0.5), r);
  const double t = e2t[k & (E2T_N - 1)];
  return ldexp(fma(t, p, t), k >> E2T_SHIFT);
}

// ------------------------------------------------------------------ NASA-7 (lane = species)
struct Thermo7 {
  double cpR, hRT, sR;
};
__device__ __forceinline__ Thermo7 nasa7_img(const MechView& V, int k, double T, double lnT, double invT) {
  const int KKp = V.KKp;
  const double* t = V.th() + k;
  // both ranges are loaded (independent LDS reads) and selected, instead of a load that waits
  // for the T_mid comparison
  const bool hi = T > t[0];
  double a[7];
#pragma unroll
  for (int c = 0; c < 7; ++c) a[c] = hi ? t[(8 + c) * KKp] : t[(1 + c) * KKp];
  const double a0 = a[0], a1 = a[1], a2 = a[2], a3 = a[3], a4 = a[4], a5 = a[5], a6 = a[6];
  // Horner forms with the 1/2 ... 1/5 factors as multiplications (no FP64 divisions)
  Thermo7 r;
  r.cpR = fma(T, fma(T, fma(T, fma(T, a4, a3), a2), a1), a0);
  r.hRT = fma(T, fma(T, fma(T, fma(T, a4 * 0.2, a3 * 0.25), a2 * (1.0 / 3.0)), a1 * 0.5), a0) + a5 * invT;
  r.sR = fma(a0, lnT, fma(T, fma(T, fma(T, fma(T, a4 * 0.25, a3 * (1.0 / 3.0)), a2 * 0.5), a1), a6));
  return r;
}

// ------------------------------------------------------------------ one reaction
struct Rxn {
  double kf, kr, mfac, pf, pr, dlkf, dlkr;
};

// Rate coefficients and concentration products of reaction slot i at (T, C).  C, gRT, hRT
// and Mg are LDS arrays of the calling wave.  Same arithmetic as oracle/ckoracle.c
// eval_reaction() (standard Chemkin-II gas kinetics: Arrhenius, third body, Lindemann /
// Troe / SRI falloff, reverse rates from equilibrium or explicit REV parameters).
// PLOG = false compiles the mechanism-without-PLOG kernels exactly as before PLOG existed (the
// PLOG branch costs 2-4 % of rate throughput in register allocation even when never taken).
// PRE: the Arrhenius parameters come in as pA (lnA, beta, Ea), loaded ahead by the caller.
template <bool PLOG = false, bool PRE = false>
__device__ __forceinline__ Rxn eval_rxn_img(const MechView& V, int i, uint32_t inf, uint32_t rs, uint32_t ps,
                                            uint32_t nuw, double T, double lnT, double invT, double lnPRT, double P,
                                            const double* C, const double* gRT, const double* hRT, const double* Mg,
                                            bool need_h, int pslot = -1, double plnf = 0.0, double gfac = 1.0,
                                            const double* pA = nullptr) {
  constexpr double INV_LN10 = 0.43429448190325176;
  const int type = rx_type(inf);
  // pslot / plnf: per-reactor A-factor perturbation (brute-force sensitivity)
  const double lnA = (PRE ? pA[0] : V.lnA()[i]) + (i == pslot ? plnf : 0.0);
  const double b = PRE ? pA[1] : V.beta()[i], Ea = PRE ? pA[2] : V.Ea()[i];
  double lnkinf = lnA + b * lnT - Ea * invT;
  double dlkf = (b + Ea * invT) * invT;
  double t13 = 0.0, t23 = 0.0;  // Landau-Teller T^(-1/3), T^(-2/3)
  if constexpr (PLOG) {
    if (type == 3 && (inf & RX_ALT)) {
      // Chebyshev (lnA, b, Ea of the slot are 0): log10 k = sum_t sum_p a[t][p] T_t(Tr) T_p(Pr),
      // Tr, Pr the reduced 1/T and log10 P; same arithmetic as oracle/ckoracle.c cheb_rate()
      const double* pt = V.aux() + AUXW * rx_aux(inf);
      const int nt = (int)pt[0], npr = (int)pt[1];
      const double Tr = (2.0 * invT - pt[2] - pt[3]) / (pt[3] - pt[2]);
      const double Pr = (2.0 * log10(P) - pt[4] - pt[5]) / (pt[5] - pt[4]);
      const double* a = pt + 6;
      double lk = 0.0, dl = 0.0;
      double tm2 = 1.0, tm1 = Tr, dm2 = 0.0, dm1 = 1.0;  // T_{t-2}, T_{t-1} and derivatives
      for (int t = 0; t < nt; ++t) {
        double tt, dt;
        if (t == 0) { tt = 1.0; dt = 0.0; }
        else if (t == 1) { tt = Tr; dt = 1.0; }
        else {
          tt = 2.0 * Tr * tm1 - tm2;
          dt = 2.0 * tm1 + 2.0 * Tr * dm1 - dm2;
          tm2 = tm1, tm1 = tt, dm2 = dm1, dm1 = dt;
        }
        double row = 0.0, p0 = 1.0, p1 = Pr;
        for (int p = 0; p < npr; ++p) {
          const double tp = p == 0 ? 1.0 : (p == 1 ? Pr : 2.0 * Pr * p1 - p0);
          if (p >= 2) p0 = p1, p1 = tp;
          row += a[t * npr + p] * tp;
        }
        lk += tt * row;
        dl += dt * row;
      }
      constexpr double LN10 = 2.302585092994046;
      lnkinf += lk * LN10;
      dlkf = dl * LN10 * (-2.0 * invT * invT / (pt[3] - pt[2]));
    } else if (type == 0 && (inf & RX_ALT)) {
      // Landau-Teller: + B T^(-1/3) + C T^(-2/3) (aux record [0], [1])
      const double* lt = V.aux() + AUXW * rx_aux(inf);
      t13 = fexp(lnT * (-1.0 / 3.0), V.e2t());
      t23 = t13 * t13;
      lnkinf += lt[0] * t13 + lt[1] * t23;
      dlkf -= (lt[0] * t13 + 2.0 * lt[1] * t23) * (1.0 / 3.0) * invT;
    } else if (type == 3) {
      // PLOG (lnA, b, Ea of the slot are 0): ln k linear in ln P between the bracketing table
      // pressures, clamped outside; aux stream = npts, then (ln P, ln A, b, E/R) per point.
      // Same arithmetic as oracle/ckoracle.c plog_rate().
      const double* pt = V.aux() + AUXW * rx_aux(inf);
      const int n = (int)pt[0];
      const double lnP = log(P);
      int j = 0;
      while (j < n - 2 && lnP > pt[1 + 4 * (j + 1)]) ++j;
      const double* t0 = pt + 1 + 4 * j;
      const double lk0 = t0[1] + t0[2] * lnT - t0[3] * invT;
      const double dk0 = (t0[2] + t0[3] * invT) * invT;
      double lk = lk0, dk = dk0;
      if (n > 1) {
        const double* t1 = t0 + 4;
        const double lk1 = t1[1] + t1[2] * lnT - t1[3] * invT;
        const double dk1 = (t1[2] + t1[3] * invT) * invT;
        const double w = fmin(fmax((lnP - t0[0]) / (t1[0] - t0[0]), 0.0), 1.0);
        lk = lk0 + w * (lk1 - lk0);
        dk = dk0 + w * (dk1 - dk0);
      }
      lnkinf += lk;
      dlkf = dk;
    }
  }
  const double* e2t = V.e2t();
  const double kf_inf = fexp(lnkinf, e2t);
  double kf = kf_inf;
  double mfac = 1.0;
  const double* ax = V.aux() + AUXW * rx_aux(inf);
  if (PLOG ? (type == 1 || type == 2) : type != 0) {
    const int tb = V.tb()[i];
    const double Mc = tb >= 0 ? Mg[tb] : C[-tb - 2];
    if (type == 1) {
      mfac = Mc;
    } else {
      // Pr = k0 [M] / k_inf from the Arrhenius exponents (one exp, no division)
      // chemically activated (extended variant, info bit 13): the slot's Arrhenius is k0 and the
      // aux record holds HIGH (k_inf), so Pr = k0 [M] / k_inf and k = k0 F / (1 + Pr)
      const bool ca = PLOG && (inf & 0x2000u);
      const double lnlim = ax[0] + ax[1] * lnT - ax[2] * invT;
      const double lnPr = (ca ? lnkinf - lnlim : lnlim - lnkinf) + log(Mc > 1e-300 ? Mc : 1e-300);
      const double Pr = fexp(lnPr, e2t);
      const double lPr = fmax(lnPr * INV_LN10, -300.0);  // log10(max(Pr, 1e-300))
      double F = 1.0;
      const int ft = rx_ftype(inf);
      if (ft == 2 || ft == 3) {
        const double fa = ax[3];
        double Fcent = (1.0 - fa) * fexp(-T * ax[4], e2t) + fa * fexp(-T * ax[5], e2t);
        if (ft == 3) Fcent += fexp(-ax[6] * invT, e2t);
        const double lnFc = log(Fcent > 1e-300 ? Fcent : 1e-300);
        const double lFc = lnFc * INV_LN10;
        const double c = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;
        const double f1 = (lPr + c) / (nn - 0.14 * (lPr + c));
        F = fexp(lnFc / (1.0 + f1 * f1), e2t);  // 10^(log10 Fcent / (1 + f1^2))
      } else if (ft == 4) {
        const double X = 1.0 / (1.0 + lPr * lPr);
        F = ax[6] * pow(ax[3] * exp(-ax[4] * invT) + exp(-T * ax[5]), X) * pow(T, ax[7]);
      }
      kf = ca ? kf_inf * (1.0 / (1.0 + Pr)) * F : kf_inf * (Pr / (1.0 + Pr)) * F;
    }
  }
  double kr = 0.0, dlkr = 0.0;
  const int r0 = sp_of(rs, 0), r1 = sp_of(rs, 1), r2 = sp_of(rs, 2), r3 = sp_of(rs, 3);
  const int p0 = sp_of(ps, 0), p1 = sp_of(ps, 1), p2 = sp_of(ps, 2), p3 = sp_of(ps, 3);
  // slots 2 and 3 hold the dummy species (C = 1, g = h = 0) unless some lane of the wave has a
  // third molecule on a side: reactions are ordered so that most strips have none, and those
  // skip 8 gathers as a wave; the results are bitwise those of the full four-slot forms
  const bool s23 = __ballot(rx_nr(inf) > 2 || rx_np(inf) > 2) != 0;
  if (rx_rev(inf)) {
    if (rx_hasrev(inf)) {
      const bool rlt = PLOG && type == 0 && (inf & RX_ALT);  // RLT terms of the explicit reverse rate
      kr = fexp(ax[8] + ax[9] * lnT - ax[10] * invT + (rlt ? ax[3] * t13 + ax[4] * t23 : 0.0), e2t);
      if (type == 2) kr *= kf / kf_inf;
      dlkr = (ax[9] + ax[10] * invT) * invT - (rlt ? (ax[3] * t13 + 2.0 * ax[4] * t23) * (1.0 / 3.0) * invT : 0.0);
    } else {
      // unit-coefficient slots: sum_products g - sum_reactants g, dnu = np - nr
      double gp = gRT[p0] + gRT[p1], gr = gRT[r0] + gRT[r1];
      if (s23) {
        gp += gRT[p2] + gRT[p3];
        gr += gRT[r2] + gRT[r3];
      }
      const double dG = gp - gr;
      const int dnu = rx_np(inf) - rx_nr(inf);
      kr = kf * fexp(dG - dnu * lnPRT, e2t);
      if (need_h) {
        const double dH = (hRT[p0] + hRT[p1]) + (hRT[p2] + hRT[p3]) - ((hRT[r0] + hRT[r1]) + (hRT[r2] + hRT[r3]));
        dlkr = dlkf - (dH - dnu) * invT;
      }
    }
  }
  double pf = C[r0] * C[r1], pr = C[p0] * C[p1];
  if (s23) {
    pf *= C[r2] * C[r3];
    pr *= C[p2] * C[p3];
  }
  Rxn e;
  e.kf = kf * gfac;  // GFAC scales forward and reverse rates alike
  e.kr = kr * gfac;
  e.mfac = mfac;
  e.pf = pf;
  e.pr = pr;
  e.dlkf = dlkf;
  e.dlkr = dlkr;
  return e;
}

// ------------------------------------------------------------------ general reactions
// FORD / RORD orders or non-integral stoichiometric coefficients (extended kernel variants only).
// Such a reaction keeps empty unit slots (nr = np = 0, so the unit-slot code skips it), carries
// info bit 14 and an aux stream after its own record (record rx_aux + 1 on):
//   nr, np, then (species, nu, order) for GEN_SLOTS reactant slots and GEN_SLOTS product slots.
constexpr uint32_t RX_GEN = 0x4000u;
constexpr int GEN_SLOTS = 8;                                  // species per side of a general reaction
constexpr int GEN_P = 2 + 3 * GEN_SLOTS;                        // first product slot of the aux stream
constexpr int GEN_RECORDS = (2 + 6 * GEN_SLOTS + AUXW - 1) / AUXW;  // 2 + 48 doubles in AUXW records

// C^o for a reaction order o, the rule of oracle/ckoracle.c conc_pow: exact products for
// o = 0..3; for 0 < o < 1 C^o above CONC_FLOOR and the chord CONC_FLOOR^(o-1) C below it (negative
// C included: Lipschitz through C = 0); otherwise exp(o ln C) for C > 0 and 0 for C <= 0
constexpr double CONC_FLOOR = 1e-14;       // [mol/cm3]
constexpr double LN_CONC_FLOOR = -32.236191301916641;  // ln(1e-14)
__device__ __forceinline__ double conc_pow(double c, double o, const double* e2t) {
  if (o == 1.0) return c;
  if (o == 2.0) return c * c;
  if (o == 0.0) return 1.0;
  if (o == 3.0) return c * c * c;
  if (o < 1.0 && c < CONC_FLOOR) return fexp((o - 1.0) * LN_CONC_FLOOR, e2t) * c;
  return c > 0.0 ? fexp(o * log(c), e2t) : 0.0;
}
// The Jacobian's d C^o / dC (oracle dconc_pow): the exact derivative of that rule -- the tangent
// o C^(o-1) above CONC_FLOOR, the chord's slope CONC_FLOOR^(o-1) below it
__device__ __forceinline__ double dconc_pow(double c, double o, const double* e2t) {
  if (o == 1.0) return 1.0;
  if (o == 2.0) return 2.0 * c;
  if (o == 0.0) return 0.0;
  if (o == 3.0) return 3.0 * c * c;
  if (o < 1.0) return c < CONC_FLOOR ? fexp((o - 1.0) * LN_CONC_FLOOR, e2t) : o * fexp((o - 1.0) * log(c), e2t);
  return c > 0.0 ? o * fexp((o - 1.0) * log(c), e2t) : 0.0;
}

// Rate coefficients and concentration products of general reaction slot i: the Arrhenius /
// third-body / falloff / explicit-REV part from eval_rxn_img (dummy species slots, so its
// products are 1), then K_c from the real coefficients and the products from the orders.
// Same arithmetic as oracle/ckoracle.c eval_reaction() with ford / rord.
__device__ __forceinline__ Rxn eval_gen_img(const MechView& V, int i, uint32_t inf, double T, double lnT, double invT,
                                            double lnPRT, double P, const double* C, const double* gRT,
                                            const double* hRT, const double* Mg, bool need_h, int pslot, double plnf,
                                            double gfac, const double*& g) {
  const uint32_t one = (uint32_t)(V.KKp - 1);
  const uint32_t dummy = one | (one << 8) | (one << 16) | (one << 24);
  const uint32_t inf2 = rx_hasrev(inf) ? inf : (inf & ~4u);  // K_c-based reverse rate: below
  Rxn e = eval_rxn_img<true>(V, i, inf2, dummy, dummy, 0u, T, lnT, invT, lnPRT, P, C, gRT, hRT, Mg, false, pslot, plnf,
                             gfac);
  g = V.aux() + AUXW * (rx_aux(inf) + 1);
  const double* e2t = V.e2t();
  const int nr = (int)g[0], np = (int)g[1];
  double pf = 1.0, pr = 1.0, dG = 0.0, dH = 0.0, dnu = 0.0;
#pragma unroll
  for (int u = 0; u < GEN_SLOTS; ++u) {
    if (u < nr) {
      const int k = (int)g[2 + 3 * u];
      const double nu = g[3 + 3 * u];
      pf *= conc_pow(C[k], g[4 + 3 * u], e2t);
      dG -= nu * gRT[k];
      if (need_h) dH -= nu * hRT[k];
      dnu -= nu;
    }
    if (u < np) {
      const int k = (int)g[GEN_P + 3 * u];
      const double nu = g[GEN_P + 1 + 3 * u];
      pr *= conc_pow(C[k], g[GEN_P + 2 + 3 * u], e2t);
      dG += nu * gRT[k];
      if (need_h) dH += nu * hRT[k];
      dnu += nu;
    }
  }
  if (rx_rev(inf) && !rx_hasrev(inf)) {
    e.kr = e.kf * fexp(dG - dnu * lnPRT, e2t);  // e.kf carries GFAC already
    e.dlkr = need_h ? e.dlkf - (dH - dnu) * invT : 0.0;
  }
  e.pf = pf;
  e.pr = pr;
  return e;
}

}  // namespace ckmi
