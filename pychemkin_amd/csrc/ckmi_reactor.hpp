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
//   VGPRs         the LU rows of M = I - gamma J (row-per-lane, N doubles per lane),
//   LDS           J (n x ld doubles, reused across steps), concentrations, g/RT, h/RT,
//                 production and dwdot/dT accumulators, third-body sums.
#pragma once
#include "ckmi_device.hpp"
#include "../../include/ckmi.h"

namespace ckmi {

constexpr int QMAX = 5;
constexpr double ETAMX1 = 10000.0, ETAMX2 = 10.0, ETAMX3 = 10.0, ETAMXF = 0.2, ETAMIN = 0.1, ETACF = 0.25;
constexpr double ADDON = 1e-6, BIAS1 = 6.0, BIAS2 = 6.0, BIAS3 = 10.0, ONEPSM = 1.000001;
constexpr int SMALL_NST = 10, MXNCF = 10, MXNEF = 7, MXNEF1 = 3, SMALL_NEF = 2, LONG_WAIT = 10, MAXCOR = 3;
constexpr double CRDOWN = 0.3, DGMAX = 0.3, RDIV = 2.0, THRESH = 1.5, CORTES = 0.1;
constexpr int MSBP = 20, MSBJ = 50;
constexpr double UROUND = 2.220446049250313e-16, NNEG_TOL = 0.01;

struct Lds {
  double* J;
  double* A;  // LU factors of I - gamma J
  double* C;
  double* gRT;
  double* hRT;
  double* wdot;
  double* dwdT;
  double* ek;
  double* Mg;
};

struct RunCtx {
  int conp, energy;
  double rho0, V0, P0;
  const ckmi_reactor_cfg* cfg;
};

__device__ __forceinline__ void profile_eval(const ckmi_reactor_cfg* c, int nprof, double t, double base, double& v,
                                             double& dvdt) {
  if (nprof <= 0) { v = base; dvdt = 0.0; return; }
  const double x0 = c->prof_t[0];
  if (t <= x0) { v = c->prof_v[0]; dvdt = 0.0; return; }
  if (t >= c->prof_t[nprof - 1]) { v = c->prof_v[nprof - 1]; dvdt = 0.0; return; }
  int j = 0;
  while (j < nprof - 2 && t >= c->prof_t[j + 1]) ++j;
  const double s = (c->prof_v[j + 1] - c->prof_v[j]) / (c->prof_t[j + 1] - c->prof_t[j]);
  v = c->prof_v[j] + s * (t - c->prof_t[j]);
  dvdt = s;
}

// J[1+k][1+j] += nu_k * dq * W_k / W_j for all participants k of one reaction
__device__ __forceinline__ void jac_scatter(const MechDev& M, const Lds& L, int ld, int nr, int np, const int4& rs,
                                            const int4& ps, const double (&rn)[SLOTS], const double (&pn)[SLOTS],
                                            int j, double dq) {
  const double wj = M.rwt[j];
#pragma unroll
  for (int u = 0; u < SLOTS; ++u) {
    if (u < nr) {
      const int k = slot(rs, u);
      atomicAdd(&L.J[(1 + k) * ld + 1 + j], -rn[u] * dq * M.wt[k] * wj);
    }
    if (u < np) {
      const int k = slot(ps, u);
      atomicAdd(&L.J[(1 + k) * ld + 1 + j], pn[u] * dq * M.wt[k] * wj);
    }
  }
}

// Right-hand side f(t, y) (returned per lane) and, if WITH_J, the approximate analytic
// Jacobian into L.J (row-major, leading dimension ld).  Mirrors oracle reactor_rhs().
template <bool WITH_J>
__device__ __forceinline__ double reactor_rhs(const MechDev& M, const RunCtx& R, double t, double yl, const Lds& L, int lane, int n,
                              int ld) {
  const int KK = M.KK;
  const bool isp = lane >= 1 && lane <= KK;
  const int s = isp ? lane - 1 : 0;
  const double T = bcast(yl, 0);
  const double Yk = isp ? yl : 0.0;
  const double rw = isp ? M.rwt[s] : 0.0;
  const double Wk = isp ? M.wt[s] : 0.0;
  const double Wbar = 1.0 / wave_sum(Yk * rw);
  const int conp = R.conp;
  double rho, P, V, dVdt = 0.0, dPdt = 0.0;
  if (conp) {
    profile_eval(R.cfg, R.cfg->nprof, t, R.P0, P, dPdt);
    rho = P * Wbar / (RU * T);
    V = R.rho0 * R.V0 / rho;
  } else {
    profile_eval(R.cfg, R.cfg->nprof, t, R.V0, V, dVdt);
    rho = R.rho0 * R.V0 / V;
    P = rho * RU * T / Wbar;
  }
  const double lnT = log(T), invT = 1.0 / T, lnPRT = log(PATM / (RU * T));
  const double Ck = rho * Yk * rw;
  SpThermo th;
  th.cpR = th.hRT = th.sR = 0.0;
  if (isp) {
    th = nasa7(M, s, T, lnT);
    L.C[s] = Ck;
    L.gRT[s] = th.hRT - th.sR;
    L.wdot[s] = 0.0;
    if (WITH_J) {
      L.hRT[s] = th.hRT;
      L.dwdT[s] = 0.0;
    }
  }
  const double Ctot = wave_sum(Ck);
  if (WITH_J) {
    for (int idx = lane; idx < n * ld; idx += WAVE) L.J[idx] = 0.0;
  }
  __syncthreads();
  for (int g = lane; g < M.G; g += WAVE) {
    double m = Ctot;
    for (int p = M.gptr[g]; p < M.gptr[g + 1]; ++p) m += M.geff[p] * L.C[M.gsp[p]];
    L.Mg[g] = m;
  }
  __syncthreads();
  const int IIp = M.IIpad;
  for (int base = 0; base < IIp; base += WAVE) {
    const int i = base + lane;
    const int nrp = M.nrp[i];
    const int nr = nrp & 0xff, np = nrp >> 8;
    if (nr + np == 0) continue;
    const RxnEval e = eval_rxn(M, i, T, lnT, invT, lnPRT, L.C, L.gRT, L.hRT, L.Mg, WITH_J);
    const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
    const int4 rs = M.rsp[i], ps = M.psp[i];
    double rn[SLOTS], pn[SLOTS];
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      rn[u] = M.rnu[u * IIp + i];
      pn[u] = M.pnu[u * IIp + i];
    }
#pragma unroll
    for (int u = 0; u < SLOTS; ++u) {
      if (u < nr) atomicAdd(&L.wdot[slot(rs, u)], -rn[u] * q);
      if (u < np) atomicAdd(&L.wdot[slot(ps, u)], pn[u] * q);
    }
    if (WITH_J) {
      double dqdT = e.mfac * (e.kf * e.dlkf * e.pf - e.kr * e.dlkr * e.pr);
      if (conp) {
        dqdT -= e.mfac * (M.ordf[i] * e.kf * e.pf - M.ordr[i] * e.kr * e.pr) * invT;
        if ((M.flags[i] & 3) == 1) dqdT -= q * invT;
      }
#pragma unroll
      for (int u = 0; u < SLOTS; ++u) {
        if (u < nr) atomicAdd(&L.dwdT[slot(rs, u)], -rn[u] * dqdT);
        if (u < np) atomicAdd(&L.dwdT[slot(ps, u)], pn[u] * dqdT);
      }
      // dq/dC_j for every reactant slot (forward) and product slot (reverse), scattered
      // into the rows of all participating species
#pragma unroll
      for (int sl = 0; sl < SLOTS; ++sl) {
        if (sl < nr && e.kf != 0.0) {
          double d = rn[sl] * powi_nu(L.C[slot(rs, sl)], rn[sl] - 1.0);
#pragma unroll
          for (int u = 0; u < SLOTS; ++u)
            if (u < nr && u != sl) d *= powi_nu(L.C[slot(rs, u)], rn[u]);
          jac_scatter(M, L, ld, nr, np, rs, ps, rn, pn, slot(rs, sl), e.mfac * e.kf * d);
        }
        if (sl < np && e.kr != 0.0) {
          double d = pn[sl] * powi_nu(L.C[slot(ps, sl)], pn[sl] - 1.0);
#pragma unroll
          for (int u = 0; u < SLOTS; ++u)
            if (u < np && u != sl) d *= powi_nu(L.C[slot(ps, u)], pn[u]);
          jac_scatter(M, L, ld, nr, np, rs, ps, rn, pn, slot(ps, sl), -e.mfac * e.kr * d);
        }
      }
    }
  }
  __syncthreads();
  const double rinv = 1.0 / rho;
  const double fY = isp ? L.wdot[s] * Wk * rinv : 0.0;
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
    else fT -= P * dVdt / (V * rho * cpm);
    if (lane == 0) fl = fT;
    if (WITH_J) {
      const double JkT = isp ? L.dwdT[s] * Wk * rinv + (conp ? fY * invT : 0.0) : 0.0;
      if (isp) {
        L.J[(1 + s) * ld] = JkT;
        L.ek[s] = ek;
      }
      __syncthreads();
      if (isp) {
        double acc = 0.0;
        for (int k = 0; k < KK; ++k) acc += L.ek[k] * L.J[(1 + k) * ld + 1 + s];
        L.J[1 + s] = -acc / cpm - fT * ck / cpm;
      }
      const double s2 = wave_sum(ck * fY + ek * JkT);
      if (lane == 0) L.J[0] = -s2 / cpm;
    }
  } else {
    if (lane == 0) fl = 0.0;
    if (WITH_J && isp) L.J[(1 + s) * ld] = L.dwdT[s] * Wk * rinv + (conp ? fY * invT : 0.0);
  }
  if (WITH_J) __syncthreads();
  return fl;
}

// ----------------------------------------------------------------- LDS LU
// Row-per-lane LU with partial pivoting of the n x n matrix A (LDS, row-major, odd leading
// dimension ld so that lane i's row accesses are bank-conflict free).  Lane i owns row i.
// Pivot rows are chosen by a wave arg-max; rows are never moved: the permutation is kept as
// (pivot step of each lane = `order`, pivot lane of step k in lane k = `permv`).
__device__ __forceinline__ bool lu_factor_lds(double* A, int ld, int lane, int n, int& order, int& permv,
                                              double& rdiag) {
  bool pivoted = lane >= n;
  order = pivoted ? (1 << 20) : 0;
  permv = 0;
  rdiag = 1.0;
  bool ok = true;
  double* row = A + (size_t)(lane < n ? lane : 0) * ld;
  for (int k = 0; k < n; ++k) {
    const double v = pivoted ? -1.0 : fabs(row[k]);
    const double vmax = wave_max(v);
    if (!(vmax > 0.0)) ok = false;
    const uint64_t mask = __ballot(!pivoted && v == vmax);
    const int p = uni(mask ? (int)__ffsll((unsigned long long)mask) - 1 : 0);
    const double* prow = A + (size_t)p * ld;
    const double rp = 1.0 / prow[k];
    if (lane == p) {
      pivoted = true;
      order = k;
      rdiag = rp;
    }
    if (lane == k) permv = p;
    if (!pivoted) {
      const double l = row[k] * rp;
      row[k] = l;
      for (int j = k + 1; j < n; ++j) row[j] = fma(-l, prow[j], row[j]);
    }
    __syncthreads();
  }
  return ok;
}

__device__ __forceinline__ double lu_solve_lds(const double* A, int ld, int lane, int n, int order, int permv,
                                               double rdiag, double b) {
  const double* row = A + (size_t)(lane < n ? lane : 0) * ld;
  for (int k = 0; k < n; ++k) {
    const int p = bcast(permv, k);
    const double sv = bcast(b, p);
    if (order > k && lane < n) b = fma(-row[k], sv, b);
  }
  double x = 0.0;
  for (int k = n - 1; k >= 0; --k) {
    const int p = bcast(permv, k);
    const double xk = bcast(b, p) * bcast(rdiag, p);
    if (lane == k) x = xk;
    if (order < k && lane < n) b = fma(-row[k], xk, b);
  }
  return x;
}

// uniform small-array access with runtime index (keeps the arrays in SGPRs)
template <int S>
__device__ __forceinline__ double pick(const double (&v)[S], int i) {
  double r = v[0];
#pragma unroll
  for (int k = 1; k < S; ++k) r = (i == k) ? v[k] : r;
  return r;
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
struct Bdf {
  double zn[QMAX + 1];
  double ewt, acor, tempv, ftemp, y;
};

__device__ __forceinline__ double wrms_lane(double v, double ewt, int n) {
  const double x = v * ewt;
  return sqrt(wave_sum(x * x) / n);
}

__device__ __forceinline__ void bdf_rescale(Bdf& b, BdfS& S) {
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

__device__ __forceinline__ void bdf_predict(Bdf& b, BdfS& S) {
  S.tn += S.h;
#pragma unroll
  for (int k = 1; k <= QMAX; ++k)
#pragma unroll
    for (int j = QMAX; j >= 1; --j)
      if (k <= S.q && j >= k && j <= S.q) b.zn[j - 1] += b.zn[j];
}

__device__ __forceinline__ void bdf_restore(Bdf& b, BdfS& S, double saved_t) {
  S.tn = saved_t;
#pragma unroll
  for (int k = 1; k <= QMAX; ++k)
#pragma unroll
    for (int j = QMAX; j >= 1; --j)
      if (k <= S.q && j >= k && j <= S.q) b.zn[j - 1] -= b.zn[j];
}

__device__ __forceinline__ void bdf_set(Bdf& b, BdfS& S) {
  const int q = S.q;
  double xi_inv = 1.0, xistar_inv = 1.0, alpha0 = -1.0, alpha0_hat = -1.0, hsum = S.h;
  S.l[0] = S.l[1] = 1.0;
#pragma unroll
  for (int i = 2; i <= QMAX; ++i) S.l[i] = 0.0;
  if (q > 1) {
#pragma unroll
    for (int j = 2; j < QMAX; ++j) {
      if (j < q) {
        hsum += S.tau[j - 1];
        xi_inv = S.h / hsum;
        alpha0 -= 1.0 / j;
#pragma unroll
        for (int i = QMAX; i >= 1; --i)
          if (i <= j) S.l[i] += S.l[i - 1] * xi_inv;
      }
    }
    alpha0 -= 1.0 / q;
    xistar_inv = -S.l[1] - alpha0;
    hsum += pick(S.tau, q - 1);
    xi_inv = S.h / hsum;
    alpha0_hat = -S.l[1] - xi_inv;
#pragma unroll
    for (int i = QMAX; i >= 1; --i)
      if (i <= q) S.l[i] += S.l[i - 1] * xistar_inv;
  }
  const double lq = pick(S.l, q);
  const double A1 = 1.0 - alpha0_hat + alpha0;
  const double A2 = 1.0 + q * A1;
  S.tq[2] = fabs(A1 / (alpha0 * A2));
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
    hsum += pick(S.tau, q);
    xi_inv = S.h / hsum;
    const double A5 = alpha0 - 1.0 / (q + 1);
    const double A6 = alpha0_hat - xi_inv;
    const double Cppinv = (1.0 - A6 + A5) / A2;
    S.tq[3] = fabs(Cppinv / (xi_inv * (q + 2) * A5));
  }
  S.tq[4] = CORTES / S.tq[2];
  S.rl1 = 1.0 / S.l[1];
  S.gamma = S.h * S.rl1;
  if (S.nst == 0) S.gammap = S.gamma;
  S.gamrat = (S.nst > 0) ? S.gamma / S.gammap : 1.0;
}

__device__ __forceinline__ void bdf_adjust_order(Bdf& b, BdfS& S, int deltaq) {
  const int q = S.q;
#pragma unroll
  for (int i = 0; i <= QMAX; ++i) S.l[i] = 0.0;
  S.l[2] = 1.0;
  if (deltaq == 1) {
    double alpha1 = 1.0, prod = 1.0, xiold = 1.0, alpha0 = -1.0, hsum = S.hscale;
#pragma unroll
    for (int j = 1; j < QMAX; ++j) {
      if (j < q) {
        hsum += pick(S.tau, j + 1);
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

__device__ __forceinline__ double dky0_lane(const Bdf& b, const BdfS& S, double t) {
  const double sc = (t - S.tn) / S.h;
  double v = 0.0;
#pragma unroll
  for (int j = QMAX; j >= 0; --j)
    if (j <= S.q) v = b.zn[j] + sc * v;
  return v;
}

}  // namespace ckmi
