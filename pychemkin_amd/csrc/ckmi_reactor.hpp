// ckmi_reactor.hpp -- wave-per-reactor closed homogeneous batch reactor on gfx950.
//
// Hot path of the reference's KINAll0D_Calculate (batchreactor.py:1149-1159): integrate
// dY_k/dt = wdot_k W_k / rho and the energy equation (CONP / CONV, ENERGY / given T) with a
// CVODE-style variable-order BDF (orders 1..5, Nordsieck history, modified Newton).
// The control flow is identical to the CPU oracle (oracle/ckoracle.c) so that the two
// produce the same step sequence up to floating-point rounding.
//
// Per wave (= reactor):
//   lanes 0..n-1  one state component each (lane 0 = T, lane k = Y_{k-1}),
//   VGPRs         the explicit inverse of M = I - gamma J (row-per-lane: N floats per lane, or
//                 N doubles in the FP64 form) and the per-lane BDF vectors,
//   LDS           the workgroup's mechanism image (shared), a per-wave slice of species
//                 vectors, the Nordsieck history and the integrator scalars, and one J assembly
//                 scratch per workgroup
//                 (lock-protected; Jacobian evaluations are ~2 % of the RHS calls),
//   HBM           the wave's last Jacobian (column-major), reloaded when only gamma changes.
#pragma once
#include "ckmi_device.hpp"
#include "ckmi_image.hpp"
#include "../../include/ckmi.h"

namespace ckmi {

constexpr int QMAX = 5;
constexpr double ETAMX1 = 10000.0, ETAMX2 = 10.0, ETAMX3 = 10.0, ETAMXF = 0.2, ETAMIN = 0.1, ETACF = 0.25;
constexpr double ADDON = 1e-6, BIAS1 = 6.0, BIAS2 = 6.0, BIAS3 = 10.0, ONEPSM = 1.000001;
constexpr int SMALL_NST = 10, MXNCF = 10, MXNEF = 7, MXNEF1 = 3, SMALL_NEF = 2, LONG_WAIT = 10, MAXCOR = 3;
constexpr double CRDOWN = 0.3, DGMAX = 0.3, RDIV = 2.0, THRESH = 1.5, CORTES = 0.1;
// MSBJ: Jacobian refresh after at most 15 steps (CVODE's msbj, default 51), as oracle/ckoracle.c: on the stiff
// ignition runs a fresher J saves more steps, RHS calls and Newton setups than its evaluations cost
// (scripts/solver_knobs_oracle.py, profiles/r06w_solver_knobs_oracle.log)
constexpr int MSBP = 20, MSBJ = 15;
constexpr double UROUND = 2.220446049250313e-16, NNEG_TOL = 0.01;

// Per-wave LDS slice (one reactor): concentrations, g/RT, h/RT, production and dwdot/dT
// accumulators, e_k (energy row of J), third-body sums.  Sized for KK <= 63 (VL = 64).
constexpr int VL = WAVE;
struct WaveLds {
  int base;  // LDS byte offset of the slice: C, gRT, hRT, wdot, dwdT, ek [VL] then Mg [G]
  __device__ __forceinline__ double* C() const { return lds_at<double>(base); }
  __device__ __forceinline__ double* gRT() const { return lds_at<double>(base + 8 * VL); }
  __device__ __forceinline__ double* hRT() const { return lds_at<double>(base + 16 * VL); }
  __device__ __forceinline__ double* wdot() const { return lds_at<double>(base + 24 * VL); }
  __device__ __forceinline__ double* dwdT() const { return lds_at<double>(base + 32 * VL); }
  __device__ __forceinline__ double* ek() const { return lds_at<double>(base + 40 * VL); }
  __device__ __forceinline__ double* Mg() const { return lds_at<double>(base + 48 * VL); }
};
constexpr int LDJ = WAVE + 1;  // leading dimension of the shared J scratch (odd: conflict-free columns)

struct RunCtx {
  int conp, energy;
  int pfr;                   // 1: problem 3, plug flow in x [cm] (conp = 1 as well); 2: problem 4,
                             // single-zone IC engine (V(t) from cfg->eng; conp = 0)
  double G, Pm;              // plug flow: mass flux rho0 u0, momentum constant P0 + G u0;
                             // engine: cp / cv (G) and temperature (Pm) of the initial charge (Woschni)
  int npv;     // VPRO / PPRO profile points (0 = constant V / P)
  int ntp;     // TPRO profile points (given-temperature runs, 0 = T from the state)
  int pslot;   // device slot of the reaction whose A is perturbed (-1 none), and ln(factor)
  double plnf;
  double gfac;               // GFAC
  double rho0, V0, P0;
  double mass;                       // rho0 V0 [g]
  double qloss, htc, areaq, tamb;    // QLOS [cal/s], HTC, AREAQ, TAMB
  int nq, na;                        // QPRO / AEXT profile points, 0 = constant
  const double* a_t;                 // the AEXT profile: prof2 (alone) or prof3 (beside QPRO)
  const double* a_v;
  double tsel;                       // midpoint of the current integration segment (pwl_eval)
  const ckmi_reactor_cfg* cfg;
};

constexpr double ERG_PER_CAL = 4.184e7;  // reference constants.py (JOULES_PER_CALORIE x 1e7)

// Piecewise-linear profile (x[np], y[np]) at t, constant outside [x0, x_np-1].  The linear piece
// is the one that contains tsel, the midpoint of the current integration segment (segments end at
// every breakpoint): a step that ends exactly on a breakpoint then uses the slope on its left and
// the first step after the restart the slope on its right, as an implicit method needs.
__device__ __forceinline__ void pwl_eval(const double* x, const double* y, int np, double t, double tsel, double& v,
                                         double& dvdt) {
  if (tsel <= x[0]) { v = y[0]; dvdt = 0.0; return; }
  if (tsel >= x[np - 1]) { v = y[np - 1]; dvdt = 0.0; return; }
  int j = 0;
  while (j < np - 2 && tsel >= x[j + 1]) ++j;
  const double s = (y[j + 1] - y[j]) / (x[j + 1] - x[j]);
  v = y[j] + s * (t - x[j]);
  dvdt = s;
}
// Plug flow (problem 3, oracle/ckoracle.c pfr_pressure): the pressure from the inviscid momentum
// equation P + G u = Pm (u = G R T / (P Wbar), the subsonic root), or the PPRO profile in x.
__device__ __forceinline__ double pfr_pressure(const ckmi_reactor_cfg* c, int npv, double G, double Pm, double t,
                                               double tsel, double T, double Wbar, double& dPdx) {
  if (npv > 0) {
    double P;
    pwl_eval(c->prof_t, c->prof_v, npv, t, tsel, P, dPdx);
    return P;
  }
  dPdx = 0.0;
  const double q = G * G * RU * T / Wbar;
  // past the choke point there is no subsonic root: clamped at the sonic one, and the step that
  // accepts such a state ends the run with CKMI_RUN_CHOKED
  return 0.5 * (Pm + sqrt(fmax(Pm * Pm - 4.0 * q, 0.0)));
}
// Single-zone IC engine (problem 4, oracle/ckoracle.c engine_volume): slider-crank with piston-pin
// offset e = -POLEN, the crank angle counted from the offset engine's top dead centre, clearance
// volume from the actual stroke and CMPR.  dVdt = dV/dt [cm3/s].
__device__ __forceinline__ void engine_volume(const double* e, double t, double& V, double& dVdt) {
  constexpr double PI = 3.14159265358979323846;
  const double B = e[CKMI_ENG_BORE], a = 0.5 * e[CKMI_ENG_STROKE], L = e[CKMI_ENG_LOLR] * a, ee = -e[CKMI_ENG_POLEN];
  const double Ab = 0.25 * PI * B * B;
  const double st = sqrt((L + a) * (L + a) - ee * ee), sb = sqrt((L - a) * (L - a) - ee * ee);
  const double Vc = Ab * (st - sb) / (e[CKMI_ENG_CMPR] - 1.0);
  const double omega = e[CKMI_ENG_RPM] * (2.0 * PI / 60.0);
  const double th = (e[CKMI_ENG_CA0] + 6.0 * e[CKMI_ENG_RPM] * t) * (PI / 180.0) + asin(ee / (L + a));
  const double sn = sin(th), cs = cos(th);
  const double u = a * sn - ee, r = sqrt(L * L - u * u);
  V = Vc + Ab * (st - (a * cs + r));
  dVdt = Ab * (a * sn + u * a * cs / r) * omega;
}
// Wall heat loss coefficient h A [erg/(K s)] of the ICHX correlation with the Woschni gas velocity
// (oracle/ckoracle.c engine_hA, same arithmetic; lnT is the log of the film temperature at which mu and
// lambda are evaluated): lane 1 + k holds species k (X_k, Y_k); mu by Wilke
// over the species fits of cfg->tran, lambda = 0.5 (sum X lambda + 1 / sum X / lambda).  Wave-uniform
// result; the KK^2 Wilke sum broadcasts (sqrt eta_j, W_j, X_j) lane by lane.
__device__ __forceinline__ double engine_hA(const MechView& Mv, const RunCtx& R, double T, double lnT, double P,
                                            double rho, double V, double Xk, double cpmass, bool isp, int s) {
  constexpr double PI = 3.14159265358979323846;
  const double* e = R.cfg->eng;
  const double* f = R.cfg->tran + 8 * s;
  const int KK = Mv.KK;
  const double muk = isp ? exp(fma(lnT, fma(lnT, fma(lnT, f[3], f[2]), f[1]), f[0])) : 1.0;
  const double lamk = isp ? exp(fma(lnT, fma(lnT, fma(lnT, f[7], f[6]), f[5]), f[4])) : 1.0;
  const double Wk = isp ? Mv.wt()[s] : 1.0;
  const double sk = sqrt(muk), qk = sqrt(sqrt(Wk));
  double den = 0.0;
  for (int j = 0; j < KK; ++j) {
    const double sj = bcast(sk, 1 + j), qj = bcast(qk, 1 + j), Wj = bcast(Wk, 1 + j), Xj = bcast(Xk, 1 + j);
    const double q = 1.0 + (sk / sj) * (qj / qk);
    den += Xj * q * q / sqrt(8.0 * (1.0 + Wk / Wj));
  }
  const double mum = wave_sum(isp ? Xk * muk / den : 0.0);
  const double l1 = wave_sum(isp ? Xk * lamk : 0.0), l2 = wave_sum(isp ? Xk / lamk : 0.0);
  const double lamm = 0.5 * (l1 + 1.0 / l2);
  const double B = e[CKMI_ENG_BORE], Ab = 0.25 * PI * B * B;
  const double a = 0.5 * e[CKMI_ENG_STROKE], L = e[CKMI_ENG_LOLR] * a, ee = -e[CKMI_ENG_POLEN];
  const double Vd = Ab * (sqrt((L + a) * (L + a) - ee * ee) - sqrt((L - a) * (L - a) - ee * ee));
  const double Vc = Vd / (e[CKMI_ENG_CMPR] - 1.0);
  const double Sp = 2.0 * e[CKMI_ENG_STROKE] * e[CKMI_ENG_RPM] / 60.0;
  const double vsw = e[CKMI_ENG_SWIRL] * e[CKMI_ENG_RPM] * (2.0 * PI / 60.0) * 0.5 * B;
  const double Pmot = R.P0 * pow(R.V0 / V, R.G);  // engine: G holds gamma of the initial charge
  const double w = (e[CKMI_ENG_C11] + e[CKMI_ENG_C12] * vsw / Sp) * Sp +
                   e[CKMI_ENG_C2] * Vd * R.Pm / (R.P0 * R.V0) * fmax(P - Pmot, 0.0);  // Pm: T_i
  const double Re = rho * w * B / mum, Pr = cpmass * mum / lamm;
  const double h = e[CKMI_ENG_HTA] * pow(Re, e[CKMI_ENG_HTB]) * pow(Pr, e[CKMI_ENG_HTC]) * lamm / B;
  return h * ((e[CKMI_ENG_CYBAR] + e[CKMI_ENG_PSBAR]) * Ab + PI * B * (V - Vc) / Ab);
}
// VPRO / PPRO / TPRO slot
__device__ __forceinline__ void profile_eval(const ckmi_reactor_cfg* c, int nprof, double t, double tsel, double base,
                                             double& v, double& dvdt) {
  if (nprof <= 0) { v = base; dvdt = 0.0; return; }
  pwl_eval(c->prof_t, c->prof_v, nprof, t, tsel, v, dvdt);
}
// the second profile slot (QPRO / AEXT)
__device__ __forceinline__ void profile2_eval(const ckmi_reactor_cfg* c, int np, double t, double tsel, double& v,
                                              double& dvdt) {
  pwl_eval(c->prof2_t, c->prof2_v, np, t, tsel, v, dvdt);
}

// Orders the wave's LDS accesses (LDS operations of one wave complete in issue order, so
// a compiler fence is all that is needed between a lane's store and another lane's load).
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// J[1+k][1+j] += (+/-) dq W_k / W_j for every (unit-coefficient) slot k of one reaction
// (column-major shared scratch Jsh[col * LDJ + row]).
__device__ __forceinline__ void jac_scatter(const MechView& V, int oJ, int nr, int np, uint32_t rs, uint32_t ps,
                                            int j, double dq) {
  double* col = lds_at<double>(oJ) + (1 + j) * LDJ + 1;
  const double dqw = dq * V.rwt()[j];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    if (u < nr) {
      const int k = sp_of(rs, u);
      atomicAdd(&col[k], -dqw * V.wt()[k]);
    }
    if (u < np) {
      const int k = sp_of(ps, u);
      atomicAdd(&col[k], dqw * V.wt()[k]);
    }
  }
}

// Jacobian terms of a general reaction (FORD / RORD / non-integral coefficients): dwdot/dT and
// dq/dC_j through the orders, scattered with the real coefficients (oracle reactor_rhs).
__device__ __noinline__ void gen_jac_terms(const MechView& V, const RunCtx& R, int i, uint32_t inf, double T,
                                           double lnT, double invT, double lnPRT, double P, const double* C,
                                           const WaveLds& L, int oJ, int conp) {
  const double* g;
  const Rxn e = eval_gen_img(V, i, inf, T, lnT, invT, lnPRT, P, C, L.gRT(), L.hRT(), L.Mg(), true, R.pslot, R.plnf,
                             R.gfac, g);
  const double* e2t = V.e2t();
  const int nr = (int)g[0], np = (int)g[1];
  const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
  double dqdT = e.mfac * (e.kf * e.dlkf * e.pf - e.kr * e.dlkr * e.pr);
  if (conp) {
    double of = 0.0, orr = 0.0;
    for (int u = 0; u < nr; ++u) of += g[4 + 3 * u];
    for (int u = 0; u < np; ++u) orr += g[GEN_P + 2 + 3 * u];
    dqdT -= e.mfac * (of * e.kf * e.pf - orr * e.kr * e.pr) * invT;
    if (rx_type(inf) == 1) dqdT -= q * invT;
  }
  for (int u = 0; u < nr; ++u) atomicAdd(&L.dwdT()[(int)g[2 + 3 * u]], -g[3 + 3 * u] * dqdT);
  for (int u = 0; u < np; ++u) atomicAdd(&L.dwdT()[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * dqdT);
  for (int side = 0; side < 2; ++side) {
    const int ns = side == 0 ? nr : np;
    const double* sl = g + (side == 0 ? 2 : GEN_P);
    const double kk = side == 0 ? e.mfac * e.kf : -e.mfac * e.kr;
    if (kk == 0.0) continue;
    for (int s = 0; s < ns; ++s) {
      const int j = (int)sl[3 * s];
      double d = dconc_pow(C[j], sl[3 * s + 2], e2t);
      for (int u = 0; u < ns; ++u)
        if (u != s) d *= conc_pow(C[(int)sl[3 * u]], sl[3 * u + 2], e2t);
      const double dqw = kk * d * V.rwt()[j];
      double* col = lds_at<double>(oJ) + (1 + j) * LDJ + 1;
      for (int u = 0; u < nr; ++u) atomicAdd(&col[(int)g[2 + 3 * u]], -g[3 + 3 * u] * dqw * V.wt()[(int)g[2 + 3 * u]]);
      for (int u = 0; u < np; ++u) atomicAdd(&col[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * dqw * V.wt()[(int)g[GEN_P + 3 * u]]);
    }
  }
}

// Right-hand side f(t, y) (one component per lane, lane 0 = T) and, if with_j, the
// approximate analytic Jacobian into the workgroup's shared J scratch (column-major, the
// caller holds its lock).  Same formulation as oracle/ckoracle.c reactor_rhs().  with_j is a
// run-time (wave-uniform) flag and the Jacobian terms are a second pass over the reactions,
// so the integrator has a single RHS call site and the register peak is that of one pass.
// PF: plug flow compiled in (problem 3); without it R.pfr is never read and the branches vanish
template <bool PL, bool PF>
__device__ __forceinline__ double reactor_rhs(const MechView& V, const RunCtx& R, double t, double yl,
                                              const WaveLds& L, int oJ, int lane, int ncol, bool with_j
#ifdef CKMI_PHASE_TIMERS
                                              , unsigned long long (&sub)[9]
#endif
) {
#ifdef CKMI_PHASE_TIMERS
  unsigned long long tsub = __builtin_amdgcn_s_memtime();
#define SUB_PHASE(k)                                      \
  do {                                                    \
    const unsigned long long t2 = __builtin_amdgcn_s_memtime(); \
    sub[k] += t2 - tsub;                                  \
    tsub = t2;                                            \
  } while (0)
#else
#define SUB_PHASE(k) (void)0
#endif
  const int KK = V.KK;
  const bool isp = lane >= 1 && lane <= KK;
  const int s = isp ? lane - 1 : 0;
  double T = bcast(yl, 0), dTdt_given = 0.0;
  if (R.ntp > 0) profile_eval(R.cfg, R.ntp, t, R.tsel, T, T, dTdt_given);  // TPRO: T(t) is given
  const double Yk = isp ? yl : 0.0;
  const double rw = isp ? V.rwt()[s] : 0.0;
  const double Wk = isp ? V.wt()[s] : 0.0;
  const double sumYW = wave_sum(Yk * rw);
  const double Wbar = 1.0 / sumYW;
  const int conp = R.conp;
  const bool pfr = PF && R.pfr == 1;
  const bool eng = PF && R.pfr == 2;
  double rho, P, V_, dVdt = 0.0, dPdt = 0.0;
  if (eng) {
    engine_volume(R.cfg->eng, t, V_, dVdt);
    rho = R.rho0 * R.V0 / V_;
    P = rho * RU * T / Wbar;
  } else if (pfr) {
    double dPdx;
    P = pfr_pressure(R.cfg, R.npv, R.G, R.Pm, t, R.tsel, T, Wbar, dPdx);
    rho = P * Wbar / (RU * T);
    V_ = R.G / rho;  // the local velocity
    dPdt = V_ * dPdx;
  } else if (conp) {
    profile_eval(R.cfg, R.npv, t, R.tsel, R.P0, P, dPdt);
    rho = P * Wbar / (RU * T);
    V_ = R.rho0 * R.V0 / rho;
  } else {
    profile_eval(R.cfg, R.npv, t, R.tsel, R.V0, V_, dVdt);
    rho = R.rho0 * R.V0 / V_;
    P = rho * RU * T / Wbar;
  }
  const double lnT = log(T), invT = 1.0 / T, lnPRT = LN_PATM_RU - lnT;
  const double Ck = rho * Yk * rw;
  Thermo7 th;
  th.cpR = th.hRT = th.sR = 0.0;
  double* C = L.C();
  if (isp) {
    th = nasa7_img(V, s, T, lnT, invT);
    C[s] = Ck;
    L.gRT()[s] = th.hRT - th.sR;
    L.wdot()[s] = 0.0;
    L.hRT()[s] = th.hRT;
    L.dwdT()[s] = 0.0;
  } else if (lane == 0) {  // the dummy slot of the unit-coefficient reaction tables
    C[SP_ONE] = 1.0;
    L.gRT()[SP_ONE] = 0.0;
    L.hRT()[SP_ONE] = 0.0;
  }
  else if (lane > KK) {
    C[lane - 1] = 0.0;  // C[KK..62] = 0: the transposed third-body table reads whole 16-row quarters
  }
  const double Ctot = rho * sumYW;  // = sum_k C_k, without a second reduction
  double* Jsh = lds_at<double>(oJ);
  if (with_j) {
    for (int idx = lane; idx < ncol * LDJ; idx += WAVE) Jsh[idx] = 0.0;
  }
  wave_lds_sync();
  // third-body concentrations [M]_g = Ctot + sum_k (eff_gk - 1) C_k, lane g
  if (V.mgt()) {
    // transposed dense table geffT[k][17] (zero rows k >= KK): lane = g + 16 q sums the species
    // quarter q, the four partials meet in the ek() scratch row (written later, in the Jacobian pass)
    const int g = lane & 15, q = lane >> 4;
    const double* e = V.geffd() + (16 * q) * 17 + g;
    const double* c = C + 16 * q;
    double m0 = 0.0, m1 = 0.0;
#pragma unroll
    for (int i = 0; i < 16; i += 2) {
      m0 = fma(e[i * 17], c[i], m0);
      m1 = fma(e[(i + 1) * 17], c[i + 1], m1);
    }
    L.ek()[lane] = m0 + m1;
    wave_lds_sync();
    if (lane < V.G) {
      const double* p = L.ek() + lane;
      L.Mg()[lane] = Ctot + ((p[0] + p[16]) + (p[32] + p[48]));
    }
  } else {
    for (int g = lane; g < V.G; g += WAVE) {
      double m = Ctot;
      for (int p = V.gptr()[g]; p < V.gptr()[g + 1]; ++p) m += V.geff()[p] * C[V.gsp()[p]];
      L.Mg()[g] = m;
    }
  }
  wave_lds_sync();
  SUB_PHASE(0);
  const int IIp = V.IIp;
  for (int base = 0; base < IIp; base += WAVE) {
    const int i = base + lane;
    const uint32_t inf = V.info()[i];
    const int nr = rx_nr(inf), np = rx_np(inf);
    if constexpr (PL) {
      if (inf & RX_GEN) {  // FORD / RORD / non-integral coefficients: real nu and orders
        const double* g;
        const Rxn e = eval_gen_img(V, i, inf, T, lnT, invT, lnPRT, P, C, L.gRT(), L.hRT(), L.Mg(), false, R.pslot,
                                   R.plnf, R.gfac, g);
        const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
#pragma unroll
        for (int u = 0; u < GEN_SLOTS; ++u) {
          if (u < (int)g[0]) atomicAdd(&L.wdot()[(int)g[2 + 3 * u]], -g[3 + 3 * u] * q);
          if (u < (int)g[1]) atomicAdd(&L.wdot()[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * q);
        }
      }
    }
    if (nr + np != 0) {
      const uint32_t rs = V.rsp()[i], ps = V.psp()[i], nuw = V.nu()[i];
      const Rxn e = eval_rxn_img<PL>(V, i, inf, rs, ps, nuw, T, lnT, invT, lnPRT, P, C, L.gRT(), L.hRT(), L.Mg(), false,
                                 R.pslot, R.plnf, R.gfac);
      const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
      const bool s23 = __ballot(nr > 2 || np > 2) != 0;  // wave-uniform: slots 2, 3 in use anywhere
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u >= 2 && !s23) break;
        if (u < nr) atomicAdd(&L.wdot()[sp_of(rs, u)], -q);
        if (u < np) atomicAdd(&L.wdot()[sp_of(ps, u)], q);
      }
    }
#ifdef CKMI_PHASE_TIMERS
    if (base / WAVE < 6) {
      const unsigned long long t2 = __builtin_amdgcn_s_memtime();
      sub[3 + base / WAVE] += t2 - tsub;
      tsub = t2;
    }
#endif
  }
  if (with_j) {
    for (int base = 0; base < IIp; base += WAVE) {
      const int i = base + lane;
      const uint32_t inf = V.info()[i];
      const int nr = rx_nr(inf), np = rx_np(inf);
      if constexpr (PL) {
        if (inf & RX_GEN) {
          gen_jac_terms(V, R, i, inf, T, lnT, invT, lnPRT, P, C, L, oJ, conp);
          continue;
        }
      }
      if (nr + np == 0) continue;
      const uint32_t rs = V.rsp()[i], ps = V.psp()[i], nuw = V.nu()[i];
      const Rxn e = eval_rxn_img<PL>(V, i, inf, rs, ps, nuw, T, lnT, invT, lnPRT, P, C, L.gRT(), L.hRT(), L.Mg(), true,
                                 R.pslot, R.plnf, R.gfac);
      const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
      double dqdT = e.mfac * (e.kf * e.dlkf * e.pf - e.kr * e.dlkr * e.pr);
      if (conp) {
        const int ordf = nr, ordr = np;  // unit-coefficient slots
        dqdT -= e.mfac * (ordf * e.kf * e.pf - ordr * e.kr * e.pr) * invT;
        if (rx_type(inf) == 1) dqdT -= q * invT;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < nr) atomicAdd(&L.dwdT()[sp_of(rs, u)], -dqdT);
        if (u < np) atomicAdd(&L.dwdT()[sp_of(ps, u)], dqdT);
      }
      // dq/dC_j for every reactant slot (forward) and product slot (reverse): the product of
      // the other three slots' concentrations (a species in two slots contributes twice)
      const int r0 = sp_of(rs, 0), r1 = sp_of(rs, 1), r2 = sp_of(rs, 2), r3 = sp_of(rs, 3);
      const int p0 = sp_of(ps, 0), p1 = sp_of(ps, 1), p2 = sp_of(ps, 2), p3 = sp_of(ps, 3);
      const double kf = e.mfac * e.kf, kr = -e.mfac * e.kr;
      if (e.kf != 0.0) {
        const double c0 = C[r0], c1 = C[r1], c2 = C[r2], c3 = C[r3];
        const double d[4] = {c1 * c2 * c3, c0 * c2 * c3, c0 * c1 * c3, c0 * c1 * c2};
#pragma unroll
        for (int sl = 0; sl < 4; ++sl)
          if (sl < nr) jac_scatter(V, oJ, nr, np, rs, ps, sp_of(rs, sl), kf * d[sl]);
      }
      if (e.kr != 0.0) {
        const double c0 = C[p0], c1 = C[p1], c2 = C[p2], c3 = C[p3];
        const double d[4] = {c1 * c2 * c3, c0 * c2 * c3, c0 * c1 * c3, c0 * c1 * c2};
#pragma unroll
        for (int sl = 0; sl < 4; ++sl)
          if (sl < np) jac_scatter(V, oJ, nr, np, rs, ps, sp_of(ps, sl), kr * d[sl]);
      }
    }
  }
  wave_lds_sync();
  SUB_PHASE(1);
  const double rinv = 1.0 / rho;
  const double fY = isp ? L.wdot()[s] * Wk * rinv : 0.0;
  double fl = fY;
  if (R.energy == 1) {
    const double cpk = th.cpR * RU * rw;
    const double hk = th.hRT * RU * T * rw;
    const double ck = conp ? cpk : cpk - RU * rw;
    const double ek = conp ? hk : hk - RU * T * rw;
    const double cpm = wave_sum(Yk * ck);
    const double sum = wave_sum(ek * fY);
    double fT = -sum / cpm;
    if (conp) fT += dPdt / (rho * cpm);
    else fT -= P * dVdt / (V_ * rho * cpm);
    // heat loss to the surroundings (QLOS + HTC AREAQ (T - TAMB), or the QPRO / AEXT profile),
    // per unit heat capacity of the reactor contents
    double qloss = R.qloss, area = R.areaq, dummy;
    if (R.nq > 0) profile2_eval(R.cfg, R.nq, t, R.tsel, qloss, dummy);
    if (R.na > 0) pwl_eval(R.a_t, R.a_v, R.na, t, R.tsel, area, dummy);
    const double mcp = R.mass * cpm;
    double q1 = pfr ? 0.0 : R.htc * area * ERG_PER_CAL;  // plug flow: no wall heat loss on this path
    if (eng) {  // engine wall heat transfer replaces QLOS / HTC
      q1 = 0.0;
      if (R.cfg->eng[CKMI_ENG_HTMODEL] == 1.0) {
        const double cpmass = wave_sum(Yk * cpk);
        // transport of the non-negative part of the composition (oracle engine_hA)
        const double xp = fmax(Yk, 0.0) * rw;
        // transport properties at the film temperature (T + Twall) / 2 (oracle engine_hA)
        q1 = engine_hA(V, R, T, log(0.5 * (T + R.cfg->eng[CKMI_ENG_TWALL])), P, rho, V_, xp / wave_sum(xp), cpmass,
                       isp, s);
        fT -= q1 * (T - R.cfg->eng[CKMI_ENG_TWALL]) / mcp;
      }
    } else if (!pfr) {
      fT -= (qloss * ERG_PER_CAL + q1 * (T - R.tamb)) / mcp;
    }
    if (lane == 0) fl = fT;
    if (with_j) {
      const double JkT = isp ? L.dwdT()[s] * Wk * rinv + (conp ? fY * invT : 0.0) : 0.0;
      if (isp) {
        Jsh[1 + s] = JkT;  // column 0 (d/dT), row 1+s
        L.ek()[s] = ek;
      }
      wave_lds_sync();
      if (isp) {
        const double* col = Jsh + (1 + s) * LDJ + 1;
        const double* ekv = L.ek();
        double acc = 0.0;
        for (int k = 0; k < KK; ++k) acc += ekv[k] * col[k];
        Jsh[(1 + s) * LDJ] = -acc / cpm - fT * ck / cpm;  // row 0, column 1+s
      }
      const double s2 = wave_sum(ck * fY + ek * JkT);
      if (lane == 0) Jsh[0] = -s2 / cpm - q1 / mcp;
    }
  } else {
    if (lane == 0) fl = dTdt_given;  // 0 without TPRO
    if (with_j && isp) Jsh[1 + s] = L.dwdT()[s] * Wk * rinv + (conp ? fY * invT : 0.0);
  }
  wave_lds_sync();
  if (pfr) {  // d/dx = (rho / G) d/dt (a TPRO profile is already T(x)); the Jacobian alike
    const double sx = rho / R.G;
    if (lane != 0 || R.energy == 1 || R.ntp == 0) fl *= sx;
    if (with_j) {
      for (int idx = lane; idx < ncol * LDJ; idx += WAVE) Jsh[idx] *= sx;
      wave_lds_sync();
    }
  }
  SUB_PHASE(2);
#undef SUB_PHASE
  return fl;
}

// ----------------------------------------------------------------- element projection
// Element conservation of the accepted corrector (oracle/ckoracle.c elem_project, same arithmetic): after
// an accepted step whose element content C y (C_mk = a_mk / W_k) has drifted from the reactor's initial
// content eb0 by more than PROJ_TOL rtol of the largest element content, acor moves to the nearest state on
// C y = eb0 in the mole-weighted norm (w_k = Y_k W_k: every species moves by a relative amount of the drift's
// size), with a ridge PROJ_RIDGE on the Gram matrix.  The element counts are
// the image's u64 table after e2t (byte e: element e of the mechanism's npe); the residual is one fused
// 8-value reduction per accepted step (checking only every 4th step was measured and rejected: the BDF error
// estimate then sees the 4-step correction as a periodic perturbation and the step counts blow up; oracle
// ckoracle.c PROJ_EVERY), the Gram matrix (rare: only on a step past the threshold) batches
// of 8 packed pairs.
constexpr int PROJ_MMAX = CKMI_PROJ_MMAX;
constexpr double PROJ_RIDGE = 1e-8, PROJ_TOL = 0.1;
constexpr double PROJ_TRACE = 1e-6;  // elements with at most this share of the largest content are left out
// scratch layout (doubles): packed lower-triangle Gram [0..35] (m (m + 1) / 2 + l), residual [40..47],
// multipliers [48..55]
constexpr int PROJ_SCR_RES = 40, PROJ_SCR_LAM = 48, PROJ_SCR_N = 56;
__device__ __forceinline__ const uint64_t* elem_table(const MechView& V) {
  return lds_at<const uint64_t>(V.o_e2t + 8 * E2T_N);
}
__device__ __forceinline__ double elem_coef(uint64_t cnt, double rw, int e) {
  return (double)(uint32_t)((cnt >> (8 * e)) & 0xffu) * rw;
}
// (m, l) of packed pair p (l <= m)
__device__ __forceinline__ void proj_pair(int p, int& m, int& l) {
  m = 0;
  while ((m + 1) * (m + 2) / 2 <= p) ++m;
  l = p - m * (m + 1) / 2;
}
// LDL^T of the ridged Gram matrix in place, then the multipliers (one lane / thread runs it: LDS reads
// and writes in program order; inline: a call in the persistent kernel costs its register allocation)
__device__ __forceinline__ void proj_solve_lds(double* scr, int M) {
  uint32_t live = 0u;
  for (int j = 0; j < M; ++j) {
    const int jj = j * (j + 1) / 2;
    const double gjj = scr[jj + j];
    const bool lj = gjj > 0.0;
    double dj = gjj * (1.0 + PROJ_RIDGE);
    for (int k = 0; k < j; ++k) dj -= scr[jj + k] * scr[jj + k] * scr[k * (k + 1) / 2 + k];
    dj = lj ? dj : 1.0;
    for (int i = j + 1; i < M; ++i) {
      const int ii = i * (i + 1) / 2;
      double v = scr[ii + j];
      for (int k = 0; k < j; ++k) v -= scr[ii + k] * scr[jj + k] * scr[k * (k + 1) / 2 + k];
      scr[ii + j] = lj ? v / dj : 0.0;
    }
    scr[jj + j] = dj;
    live |= (lj ? 1u : 0u) << j;
  }
  for (int j = 0; j < M; ++j) {  // forward: z in the residual slots
    double v = scr[PROJ_SCR_RES + j];
    for (int k = 0; k < j; ++k) v -= scr[j * (j + 1) / 2 + k] * scr[PROJ_SCR_RES + k];
    scr[PROJ_SCR_RES + j] = ((live >> j) & 1u) ? v : 0.0;
  }
  for (int j = M - 1; j >= 0; --j) {  // backward: lambda
    double v = scr[PROJ_SCR_RES + j] / scr[j * (j + 1) / 2 + j];
    for (int i = j + 1; i < M; ++i) v -= scr[i * (i + 1) / 2 + j] * scr[PROJ_SCR_LAM + i];
    scr[PROJ_SCR_LAM + j] = ((live >> j) & 1u) ? v : 0.0;
  }
}

// wave-per-reactor form: lane = component (zn0 its predicted value, acor its accumulated correction),
// eb0 the reactor's initial element contents (uniform, LDS), scr PROJ_SCR_N doubles of free wave-local LDS
__device__ __forceinline__ void elem_project_wave(const MechView& V, int npe, const double* eb0, double rtol,
                                                  double zn0, double& acor, int lane,
                                                  double* scr) {
  const bool isp = lane >= 1 && lane <= V.KK;
  const int s = isp ? lane - 1 : 0;
  const uint64_t cnt = isp ? elem_table(V)[s] : 0ull;
  const double rw = isp ? V.rwt()[s] : 0.0;
  const double y = zn0 + acor;
  double v[PROJ_MMAX];
#pragma unroll
  for (int e = 0; e < PROJ_MMAX; ++e) v[e] = elem_coef(cnt, rw, e) * y;
  wave_sum_multi<PROJ_MMAX>(v, lane);
  double rmax = 0.0, bmax = 0.0;
#pragma unroll
  for (int e = 0; e < PROJ_MMAX; ++e) {
    if (e < npe) {
      v[e] -= eb0[e];
      rmax = fmax(rmax, fabs(v[e]));
      bmax = fmax(bmax, eb0[e]);
    }
  }
  if (!(rmax > PROJ_TOL * rtol * bmax)) return;
  const double w = (isp && y > 0.0) ? y * V.wt()[s] : 0.0;  // moles: relative changes of the drift's size
  const int npair = npe * (npe + 1) / 2;
#pragma unroll 1
  for (int p0 = 0; p0 < npair; p0 += 8) {
    double g[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      int m, l;
      proj_pair(p0 + i, m, l);
      g[i] = p0 + i < npair ? elem_coef(cnt, rw, m) * elem_coef(cnt, rw, l) * w : 0.0;
    }
    wave_sum_multi<8>(g, lane);
    if (lane == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (p0 + i < npair) scr[p0 + i] = g[i];
    }
  }
  if (lane == 0) {
#pragma unroll
    for (int e = 0; e < PROJ_MMAX; ++e) {
      if (e < npe) {
        scr[PROJ_SCR_RES + e] = v[e];
        if (!(eb0[e] > PROJ_TRACE * bmax)) scr[e * (e + 1) / 2 + e] = 0.0;  // trace element: left out
      }
    }
    proj_solve_lds(scr, npe);
  }
  wave_lds_sync();
  double sc = 0.0;
#pragma unroll
  for (int e = 0; e < PROJ_MMAX; ++e)
    if (e < npe) sc += elem_coef(cnt, rw, e) * scr[PROJ_SCR_LAM + e];
  acor -= w * sc;
}

// ----------------------------------------------------------------- Newton matrix in VGPRs
// M = I - gamma J is held row-per-lane in registers: lane i owns row i as a[0..N-1]
// (N = compile-time padded size >= n; columns >= n are zero, lanes >= n are inert).  LU with
// partial pivoting: the pivot search is a DPP wave max, the pivot row is broadcast with
// v_readlane, rows are not moved during elimination.  Afterwards the rows are permuted with
// ds_bpermute so that lane k holds the k-th pivot row (L multipliers left of the diagonal,
// U / u_kk right of it, 1 / u_kk in rdiag): both triangular sweeps then broadcast from a
// compile-time lane and never touch LDS memory.

// The lane index laundered through an empty volatile asm: comparisons of it with the
// unrolled loop constants below must be computed where they are used.  Left visible, LICM
// hoists all N (lane == j) masks / identity entries out of the persistent reactor loop and
// keeps them live (spilled) across the whole integrator.
__device__ __forceinline__ int opaque_lane(int lane) {
  asm volatile("" : "+v"(lane));
  return lane;
}

__device__ __forceinline__ double bpermute(int src_lane, double v) {
  const int lo = __builtin_amdgcn_ds_bpermute(src_lane * 4, __double2loint(v));
  const int hi = __builtin_amdgcn_ds_bpermute(src_lane * 4, __double2hiint(v));
  return __hiloint2double(hi, lo);
}

// Two forms of the Newton matrix (kernel template parameter F64 of reactor_kernel):
//   NewtonMatrixF32S  FP64 Gauss-Jordan, inverse stored in FP32 between factorisations (N VGPRs:
//                     3 waves per SIMD); the default
//   NewtonMatrixGJ64  the same inverse kept in FP64 (2N VGPRs: 2 waves per SIMD), for tolerances
//                     tighter than an FP32-rounded inverse resolves (rtol < 1e-9, ckmi.hip)
// A factorisation in FP32 (tried, with error-weight equilibration) fails on ~6 % of the bench
// reactors (Newton convergence / error-test failures): the elimination needs FP64, the stored
// inverse does not.
constexpr int GJ_BATCH = 4;  // row pairs read per batch in the elimination (2 and 8 measured slower)
// Gauss-Jordan form: factor() overwrites a with the explicit inverse of the row-permuted
// matrix (same partial pivoting sequence as LU: the pivot of step k is the largest |a[k]|
// among the rows not yet used).  Lane p_k (permv on lane k) ends up holding row k of
// (P M)^-1, so a solve is one matrix-vector product whose 54 broadcasts are independent of
// each other -- instead of two dependent 54-step triangular sweeps.  n^3 instead of n^3/3
// FMAs at factor time, paid back within one solve (1.5 solves per factorisation on average
// is the minimum; the bench workload does 11).
template <int N>
struct NewtonMatrixGJ64 {
  double a[N];
  int permv;  // lane k: the lane whose row was the pivot of step k

  template <typename TJ>
  __device__ __forceinline__ void build(const TJ* J, int ldj, double gamma, int lane_in, int n) {
    const int lane = opaque_lane(lane_in);
#pragma unroll
    for (int j = 0; j < N; ++j)
      a[j] = (j == lane ? 1.0 : 0.0) - gamma * J[j * ldj + lane];  // J rows / columns >= n are zero
  }

  // orow: LDS byte offset of an N-double scratch row of the calling wave (16-byte aligned).
  // The pivot row is broadcast through it: the pivot lane writes its row with ds_write_b128,
  // every lane reads it back with broadcast ds_read_b128 -- 1 LDS instruction per element
  // instead of 2 v_readlane + the SGPR-forwarding wait of a register broadcast.
  __device__ __forceinline__ bool factor(int lane_in, int n, int orow) {
    const int lane = opaque_lane(lane_in);
    bool pivoted = lane >= N;
    permv = lane;
    bool ok = true;
    // laundered like the lane index: otherwise the 27 row addresses are hoisted out of the
    // reactor loop and held in VGPRs for its whole life
    double2* row = lds_at<double2>(__builtin_amdgcn_readfirstlane(opaque_lane(orow)));
    constexpr int NP = N / 2;  // row pairs (ds_read_b128)
    // partial pivoting on |a| rounded to fp32 (ties within fp32 rounding go to the lowest lane;
    // any of them is an equally good pivot).  The search for column k+1 is software-pipelined
    // into the elimination of step k: column k+1 is updated first, and the DPP stages of its
    // wave max are spread between the remaining row pairs, so their latency overlaps FMAs.
    uint32_t v0 = pivoted ? 0u : __float_as_uint((float)fabs(a[0]));
    uint32_t vmax = wave_max_u32(v0);
#pragma unroll
    for (int k = 0; k < N; ++k) {
      if (vmax == 0u) ok = false;
      const uint64_t mask = __ballot(!pivoted && v0 == vmax);
      const int p = uni(mask ? (int)__ffsll((unsigned long long)mask) - 1 : 0);
      const bool me = lane == p;
      if (me) {
        // 64-bit stores by inline asm: any register pair is a valid source, so the allocator never
        // re-packs the row into 4-VGPR tuples for ds_write_b128 (2 v_mov per processed column and
        // step: ~3,000 VALU issues per factorisation at N = 54).  LDS operations of one wave complete
        // in issue order, so the other lanes' ds_read_b128 after wave_lds_sync see these stores.
        const uint32_t rb = (uint32_t)(uintptr_t)row;
#pragma unroll
        for (int j = 0; j < N; ++j)
          asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(rb), "v"(a[j]), "i"(8 * j) : "memory");
      }
      wave_lds_sync();  // other lanes' reads must follow the pivot lane's writes
      const double piv = bcast(a[k], p);
      const double rp = rcp_nr(piv);
      if (me) pivoted = true;
      if (lane == k) permv = p;
      // row p becomes row p / piv; every other row i loses (a_i[k] / piv) x row p.  One FMA
      // form for both: g = (piv - 1) / piv on the pivot lane gives a_p - g a_p = a_p / piv.
      const double g = me ? (piv - 1.0) * rp : a[k] * rp;
      const double ak = me ? rp : -g;
      const int P0 = (k + 1 < N ? k + 1 : k) / 2;  // the pair holding column k+1 goes first
      uint32_t w = 0u;
#pragma unroll
      for (int t = 0; t < NP; ++t) {
        const int P = (P0 + t) % NP;
        const double2 r = row[P];
        if (2 * P != k) a[2 * P] = fma(-g, r.x, a[2 * P]);
        if (2 * P + 1 != k) a[2 * P + 1] = fma(-g, r.y, a[2 * P + 1]);
        if (k + 1 < N) {
          if (t == 0) {
            v0 = pivoted ? 0u : __float_as_uint((float)fabs(a[k + 1]));
            w = v0;
          }
          if (t == 2) w = max(w, (uint32_t)__builtin_amdgcn_mov_dpp((int)w, DPP_QUAD_1032, 0xf, 0xf, false));
          if (t == 5) w = max(w, (uint32_t)__builtin_amdgcn_mov_dpp((int)w, DPP_QUAD_2301, 0xf, 0xf, false));
          if (t == 8) w = max(w, (uint32_t)__builtin_amdgcn_mov_dpp((int)w, DPP_ROW_HALF_MIRROR, 0xf, 0xf, false));
          if (t == 11) w = max(w, (uint32_t)__builtin_amdgcn_mov_dpp((int)w, DPP_ROW_MIRROR, 0xf, 0xf, false));
          if (t == 14) {
            const uint32_t r0 = __builtin_amdgcn_readlane(w, 0), r1 = __builtin_amdgcn_readlane(w, 16);
            const uint32_t r2 = __builtin_amdgcn_readlane(w, 32), r3 = __builtin_amdgcn_readlane(w, 48);
            vmax = max(max(r0, r1), max(r2, r3));
          }
        }
        if (t % GJ_BATCH == GJ_BATCH - 1) asm volatile("" ::: "memory");  // row reads in flight (VGPR peak)
      }
      a[k] = ak;
    }
    return ok;
  }

  template <typename TJ>
  __device__ __forceinline__ bool build_factor(const TJ* J, int ldj, double gamma, int lane, int n, int orow) {
    build(J, ldj, gamma, lane, n);
    return factor(lane, n, orow);
  }

  // x = M^-1 b (lane k: component k)
  __device__ __forceinline__ double solve(double b, int lane_in, int n) const {
    const int lane = opaque_lane(lane_in);
    if (lane >= n) b = 0.0;
    const double bp = bpermute(permv, b);  // lane j: b[p_j]
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      s0 = fma(a[j], bcast(bp, j), s0);
      if (j + 1 < N) s1 = fma(a[j + 1], bcast(bp, j + 1), s1);
    }
    // lane p_k holds x_k; bring it to lane k
    return bpermute(permv, s0 + s1);
  }
};


// The FP64 Gauss-Jordan inverse above, stored in FP32 between factorisations: the factorisation
// itself keeps FP64 (its N doubles are live only inside ST_SETUP), the inverse that stays in
// registers across the RHS evaluations takes N VGPRs instead of 2N.
template <int N>
struct NewtonMatrixF32S {
  float a[N];
  int permv;
  template <typename TJ>
  __device__ __forceinline__ bool build_factor(const TJ* J, int ldj, double gamma, int lane, int n, int orow) {
    NewtonMatrixGJ64<N> m;
    const bool ok = m.build_factor(J, ldj, gamma, lane, n, orow);
#pragma unroll
    for (int j = 0; j < N; ++j) a[j] = (float)m.a[j];
    permv = m.permv;
    return ok;
  }
  __device__ __forceinline__ double solve(double b, int lane_in, int n) const {
    const int lane = opaque_lane(lane_in);
    if (lane >= n) b = 0.0;
    const double bp = bpermute(permv, b);
    double s0 = 0.0, s1 = 0.0;
#pragma unroll
    for (int j = 0; j < N; j += 2) {
      s0 = fma((double)a[j], bcast(bp, j), s0);
      if (j + 1 < N) s1 = fma((double)a[j + 1], bcast(bp, j + 1), s1);
    }
    return bpermute(permv, s0 + s1);
  }
};

// uniform small-array access with runtime index (keeps the arrays in SGPRs)
template <int S>
__device__ __forceinline__ double pick(const double (&v)[S], int i) {
  double r = v[0];
#pragma unroll
  for (int k = 1; k < S; ++k) r = (i == k) ? v[k] : r;
  return r;
}

// x^(1/p) for the step-size / order heuristics (eta = 1 / (BIAS * dsm)^(1/L) + ...): computed
// with the hardware f32 log2 / exp2.  The heuristic only picks the next h; its ~1e-7 relative
// error is far below anything the error test resolves, and it replaces an FP64 pow
// (~200 dependent instructions) on every step.
__device__ __forceinline__ double eta_root(double x, int p) {
  return (double)exp2f(log2f((float)x) / (float)p);
}

// ----------------------------------------------------------------- BDF state
// Uniform integrator scalars live in LDS (one copy per wave): every lane reads the same
// address (broadcast), which keeps ~60 doubles out of the SGPR file.
struct BdfS {
  double h, hscale, hprime, eta, etamax, hmax_inv, hmin, tn, rl1, gamma, gammap, gamrat, crate, acnrm, saved_tq5, hu;
  double l[QMAX + 1], tq[6], tau[QMAX + 2];
  int q, qprime, qwait, L, nst, nstlp, nstlj, jcur, ncf_tot, nef_tot, nlu, nfe, nje, nni;
  double rtol, atol;
  int nneg;
};

// per-lane vectors (VGPRs)
// The Nordsieck history lives in the wave's LDS slice (zn[j] of lane l at base_l + j * 512):
// it is touched a few times per step, and its 12 VGPRs are worth more to the register-resident
// Newton matrix.
// ST = threads per Nordsieck row: WAVE for the wave-per-reactor kernel, the workgroup size for
// the workgroup-per-reactor kernel of large mechanisms (ckmi_big.hip).
template <int ST>
struct ZnLdsT {
  int base;  // LDS byte offset of this thread's zn[0]
  __device__ __forceinline__ double& operator[](int j) const { return *lds_at<double>(base + j * ST * 8); }
};
using ZnLds = ZnLdsT<WAVE>;
constexpr int ZN_BYTES = (QMAX + 1) * WAVE * 8;

template <int ST>
struct BdfT {
  ZnLdsT<ST> zn;
  double ewt, acor, tempv, ftemp, y;
};
using Bdf = BdfT<WAVE>;

__device__ __forceinline__ double wrms_lane(double v, double ewt, int n) {
  const double x = v * ewt;
  return sqrt(wave_sum(x * x) / n);
}

template <class BB, class SS>
__device__ __forceinline__ void bdf_rescale(BB& b, SS& S) {
  double factor = S.eta;
#pragma unroll
  for (int j = 1; j <= QMAX; ++j) {
    if (j <= S.q) {
      b.zn[j] *= factor;
      factor *= S.eta;
    }
  }
  S.h = S.hscale * S.eta;
  S.hscale = S.h;
}

// zn_{j-1} += zn_j for k = 1..q, j = q..k (Pascal-triangle prediction), in registers
template <class BB, class SS>
__device__ __forceinline__ void bdf_predict(BB& b, SS& S) {
  S.tn += S.h;
  const int q = S.q;
  double z[QMAX + 1];
#pragma unroll
  for (int j = 0; j <= QMAX; ++j) z[j] = b.zn[j];
#pragma unroll
  for (int k = 1; k <= QMAX; ++k)
#pragma unroll
    for (int j = QMAX; j >= 1; --j)
      if (j >= k) z[j - 1] = (k <= q && j <= q) ? z[j - 1] + z[j] : z[j - 1];
#pragma unroll
  for (int j = 0; j < QMAX; ++j) b.zn[j] = z[j];
}

template <class BB, class SS>
__device__ __forceinline__ void bdf_restore(BB& b, SS& S, double saved_t) {
  S.tn = saved_t;
  const int q = S.q;
  double z[QMAX + 1];
#pragma unroll
  for (int j = 0; j <= QMAX; ++j) z[j] = b.zn[j];
#pragma unroll
  for (int k = 1; k <= QMAX; ++k)
#pragma unroll
    for (int j = QMAX; j >= 1; --j)
      if (j >= k) z[j - 1] = (k <= q && j <= q) ? z[j - 1] - z[j] : z[j - 1];
#pragma unroll
  for (int j = 0; j < QMAX; ++j) b.zn[j] = z[j];
}

// The coefficient recursion on locals (l[], h, tau) and one store of each result (an LDS-resident form,
// updated in place, gave bitwise the same values 0.6 % slower), CVODE's cvSetBDF; oracle set_bdf.
template <class BB, class SS>
__device__ __forceinline__ void bdf_set(BB& b, SS& S) {
  const int q = S.q;
  const double h = S.h;
  double tau[QMAX + 1];
#pragma unroll
  for (int i = 0; i <= QMAX; ++i) tau[i] = S.tau[i];
  double l[QMAX + 1];
  double xi_inv = 1.0, xistar_inv = 1.0, alpha0 = -1.0, alpha0_hat = -1.0, hsum = h;
  l[0] = l[1] = 1.0;
#pragma unroll
  for (int i = 2; i <= QMAX; ++i) l[i] = 0.0;
  if (q > 1) {
#pragma unroll
    for (int j = 2; j < QMAX; ++j) {
      if (j < q) {
        hsum += tau[j - 1];
        xi_inv = h / hsum;
        alpha0 -= 1.0 / j;
#pragma unroll
        for (int i = QMAX; i >= 1; --i)
          if (i <= j) l[i] += l[i - 1] * xi_inv;
      }
    }
    alpha0 -= 1.0 / q;
    xistar_inv = -l[1] - alpha0;
    double tq1 = tau[0];  // tau[q - 1] with a run-time q, as selects
#pragma unroll
    for (int i = 1; i <= QMAX; ++i) tq1 = (i == q - 1) ? tau[i] : tq1;
    hsum += tq1;
    xi_inv = h / hsum;
    alpha0_hat = -l[1] - xi_inv;
#pragma unroll
    for (int i = QMAX; i >= 1; --i)
      if (i <= q) l[i] += l[i - 1] * xistar_inv;
  }
  double lq = l[0];
#pragma unroll
  for (int i = 1; i <= QMAX; ++i) lq = (i == q) ? l[i] : lq;
#pragma unroll
  for (int i = 0; i <= QMAX; ++i) S.l[i] = l[i];
  const double A1 = 1.0 - alpha0_hat + alpha0;
  const double A2 = 1.0 + q * A1;
  const double tq2 = fabs(A1 / (alpha0 * A2));
  S.tq[2] = tq2;
  S.tq[5] = fabs(A2 * xistar_inv / (lq * xi_inv));
  if (S.qwait == 1) {
    if (q > 1) {
      const double Cc = xistar_inv / lq;
      const double A3 = alpha0 + 1.0 / q;
      const double A4 = alpha0_hat + xi_inv;
      const double Cpinv = (1.0 - A4 + A3) / A3;
      S.tq[1] = fabs(Cc * Cpinv);
    } else {
      S.tq[1] = 1.0;
    }
    double tq = tau[0];  // tau[q]
#pragma unroll
    for (int i = 1; i <= QMAX; ++i) tq = (i == q) ? tau[i] : tq;
    hsum += tq;
    xi_inv = h / hsum;
    const double A5 = alpha0 - 1.0 / (q + 1);
    const double A6 = alpha0_hat - xi_inv;
    const double Cppinv = (1.0 - A6 + A5) / A2;
    S.tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
  }
  S.tq[4] = CORTES / tq2;
  const double rl1 = 1.0 / l[1];
  const double gamma = h * rl1;
  S.rl1 = rl1;
  S.gamma = gamma;
  if (S.nst == 0) S.gammap = gamma;
  S.gamrat = (S.nst > 0) ? gamma / S.gammap : 1.0;
}


template <class BB, class SS>
__device__ __forceinline__ void bdf_adjust_order(BB& b, SS& S, int deltaq) {
  const int q = S.q;
#pragma unroll
  for (int i = 0; i <= QMAX; ++i) S.l[i] = 0.0;
  S.l[2] = 1.0;
  if (deltaq == 1) {
    double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = S.hscale;
#pragma unroll
    for (int j = 1; j < QMAX; ++j) {
      if (j < q) {
        hsum += S.tau[j + 1];
        const double xi = hsum / S.hscale;
        prod *= xi;
        alpha0 -= 1.0 / (j + 1);
        alpha1 += 1.0 / xi;
#pragma unroll
        for (int i = QMAX; i >= 2; --i)
          if (i <= j + 2) S.l[i] = S.l[i] * xiold + S.l[i - 1];
        xiold = xi;
      }
    }
    const double A1 = (-alpha0 - alpha1) / prod;
    const double znL = A1 * b.zn[QMAX];
#pragma unroll
    for (int j = 2; j <= QMAX; ++j)
      if (j <= q) b.zn[j] += S.l[j] * znL;
#pragma unroll
    for (int j = 1; j <= QMAX; ++j)
      if (j == q + 1) b.zn[j] = znL;
  } else {
    double hsum = 0.0;
#pragma unroll
    for (int j = 1; j <= QMAX; ++j) {
      if (j <= q - 2) {
        hsum += S.tau[j];
        const double xi = hsum / S.hscale;
#pragma unroll
        for (int i = QMAX; i >= 2; --i)
          if (i <= j + 2) S.l[i] = S.l[i] * xi + S.l[i - 1];
      }
    }
    double znq = 0.0;
#pragma unroll
    for (int j = 0; j <= QMAX; ++j)
      if (j == q) znq = b.zn[j];
#pragma unroll
    for (int j = 2; j <= QMAX; ++j)
      if (j < q) b.zn[j] -= S.l[j] * znq;
  }
}

template <class BB, class SS>
__device__ __forceinline__ double dky0_lane(const BB& b, const SS& S, double t) {
  const double sc = (t - S.tn) / S.h;
  double v = 0.0;
#pragma unroll
  for (int j = QMAX; j >= 0; --j)
    if (j <= S.q) v = b.zn[j] + sc * v;
  return v;
}

}  // namespace ckmi
