// ckmi.hip -- gfx950 kernels and the C ABI of libckmi.so (see include/ckmi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "ckmi_reactor.hpp"

using namespace ckmi;

namespace {

thread_local std::string g_err;

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_CHECK(x)                                                                   \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) return fail(CKMI_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

enum { NF_FIRST = 0, NF_CONV_FAIL = 1, NF_ERR_FAIL = 2 };
enum { CF_NONE = 0, CF_BAD_J = 1, CF_OTHER = 2 };

// ---------------------------------------------------------------- reactor kernel
template <int N>
struct Wave {
  const MechDev& M;
  const RunCtx& R;
  const Lds& L;
  int lane, n, ld;
  int order, permv;
  double rdiag;

  __device__ Wave(const MechDev& m, const RunCtx& r, const Lds& l, int lane_, int n_, int ld_)
      : M(m), R(r), L(l), lane(lane_), n(n_), ld(ld_), order(0), permv(0), rdiag(1.0) {}

  __device__ __forceinline__ double f(double t, double yl) { return reactor_rhs<false>(M, R, t, yl, L, lane, n, ld); }
  __device__ __forceinline__ double fj(double t, double yl) { return reactor_rhs<true>(M, R, t, yl, L, lane, n, ld); }

  // M = I - gamma J from the Jacobian in LDS, factored in LDS (row-per-lane)
  __device__ __forceinline__ bool build_and_factor(double gamma) {
    if (lane < n) {
      const double* jr = L.J + (size_t)lane * ld;
      double* ar = L.A + (size_t)lane * ld;
      for (int j = 0; j < n; ++j) ar[j] = (j == lane ? 1.0 : 0.0) - gamma * jr[j];
    }
    __syncthreads();
    return lu_factor_lds(L.A, ld, lane, n, order, permv, rdiag);
  }
  __device__ __forceinline__ double solve(double b) { return lu_solve_lds(L.A, ld, lane, n, order, permv, rdiag, b); }
};

template <int N>
__device__ __forceinline__ int bdf_nls(Bdf& b, BdfS& S, Wave<N>& w, int nflag) {
  const int n = w.n;
  const bool act = w.lane < n;
  int convfail = (nflag == NF_FIRST || nflag == NF_ERR_FAIL) ? CF_NONE : CF_OTHER;
  int call_setup = (nflag != NF_FIRST) || S.nst == 0 || S.nst >= S.nstlp + MSBP || fabs(S.gamrat - 1.0) > DGMAX;
  for (;;) {
    b.y = b.zn[0];
    b.ftemp = w.f(S.tn, b.y);
    S.nfe++;
    if (call_setup) {
      const double dgamma = fabs(S.gamma / S.gammap - 1.0);
      const int jbad = S.nst == 0 || S.nst >= S.nstlj + MSBJ || (convfail == CF_BAD_J && dgamma < DGMAX) ||
                       convfail == CF_OTHER;
      if (jbad) {
        (void)w.fj(S.tn, b.y);
        S.nfe++;
        S.nje++;
        S.nstlj = S.nst;
        S.jcur = 1;
      } else {
        S.jcur = 0;
      }
      const bool ok = w.build_and_factor(S.gamma);
      S.nlu++;
      S.crate = 1.0;
      S.gammap = S.gamma;
      S.gamrat = 1.0;
      S.nstlp = S.nst;
      if (!ok) return 1;
    }
    b.acor = 0.0;
    double delp = 0.0;
    int mm = 0;
    int failed = 0;
    for (;;) {
      const double rhs = act ? S.gamma * b.ftemp - (S.rl1 * b.zn[1] + b.acor) : 0.0;
      double x = w.solve(rhs);
      S.nni++;
      if (S.gamrat != 1.0) x *= 2.0 / (1.0 + S.gamrat);
      if (!act) x = 0.0;
      const double del = wrms_lane(x, b.ewt, n);
      b.acor += x;
      b.y = b.zn[0] + b.acor;
      if (mm > 0) S.crate = fmax(CRDOWN * S.crate, del / delp);
      const double dcon = del * fmin(1.0, S.crate) / S.tq[4];
      if (dcon <= 1.0) {
        if (S.nneg) {
          const bool neg = act && w.lane >= 1 && b.y < 0.0;
          const double xn = neg ? b.y * b.ewt : 0.0;
          const double s = wave_sum(xn * xn);
          if (s > 0.0) {
            if (sqrt(s / n) > NNEG_TOL) {
              failed = 2;
              break;
            }
            if (neg) {
              b.y = 0.0;
              b.acor = -b.zn[0];
            }
            S.acnrm = wrms_lane(b.acor, b.ewt, n);
            S.jcur = 0;
            return 0;
          }
        }
        S.acnrm = (mm == 0) ? del : wrms_lane(b.acor, b.ewt, n);
        S.jcur = 0;
        return 0;
      }
      mm++;
      if (mm == MAXCOR || (mm >= 2 && del > RDIV * delp)) {
        failed = 1;
        break;
      }
      delp = del;
      b.ftemp = w.f(S.tn, b.y);
      S.nfe++;
    }
    if (failed == 1 && !S.jcur) {
      convfail = CF_BAD_J;
      call_setup = 1;
      continue;
    }
    return 1;
  }
}

template <int N>
__device__ __forceinline__ double bdf_initial_step(Bdf& b, BdfS& S, Wave<N>& w, double tout) {
  const int n = w.n;
  const bool act = w.lane < n;
  const double t0 = S.tn;
  const double tdist = fabs(tout - t0);
  const double tround = UROUND * fmax(fabs(t0), fabs(tout));
  const double hlb = 100.0 * tround;
  double hub = 0.1 * tdist;
  const double num = act ? fabs(b.zn[1]) : 0.0;
  const double den = 0.1 * fabs(b.zn[0]) + S.atol;
  const double hub_inv = wave_max(act ? num / (den > 0 ? den : 1e-300) : 0.0);
  if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
  double hg = sqrt(hlb * hub);
  if (hub < hlb) return hg;
  double hnew = hg;
  for (int count = 1; count <= 4; ++count) {
    const double y1 = b.zn[0] + hg * b.zn[1];
    double f1 = w.f(t0 + hg, y1);
    S.nfe++;
    f1 = act ? (f1 - b.zn[1]) / hg : 0.0;
    const double yddnrm = wrms_lane(f1, b.ewt, n);
    hnew = (yddnrm * hub * hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * hub);
    if (count == 4) break;
    const double hrat = hnew / hg;
    if (hrat > 0.5 && hrat < 2.0) break;
    if (count >= 2 && hrat > 2.0) {
      hnew = hg;
      break;
    }
    hg = hnew;
  }
  double h0 = 0.5 * hnew;
  if (h0 < hlb) h0 = hlb;
  if (h0 > hub) h0 = hub;
  return h0;
}

template <int N>
__device__ __forceinline__ void bdf_start(Bdf& b, BdfS& S, Wave<N>& w, double t, double yl, double tout, double h0, double hmax) {
  const bool act = w.lane < w.n;
  S.tn = t;
  b.zn[0] = act ? yl : 0.0;
#pragma unroll
  for (int j = 1; j <= QMAX; ++j) b.zn[j] = 0.0;
  b.ewt = act ? 1.0 / (S.rtol * fabs(b.zn[0]) + S.atol) : 0.0;
  b.zn[1] = w.f(t, b.zn[0]);
  S.nfe++;
  if (!act) b.zn[1] = 0.0;
  double h = h0 > 0.0 ? h0 : bdf_initial_step(b, S, w, tout);
  if (h > hmax) h = hmax;
  if (h > tout - t) h = tout - t;
  b.zn[1] *= h;
  S.h = S.hscale = S.hprime = h;
  S.q = S.qprime = 1;
  S.L = 2;
  S.qwait = S.L;
  S.etamax = ETAMX1;
  S.nst = 0;
  S.nstlp = 0;
  S.nstlj = 0;
  S.jcur = 0;
  S.crate = 1.0;
  S.gammap = S.gamma = S.h;
  S.gamrat = 1.0;
  S.saved_tq5 = 0.0;
#pragma unroll
  for (int i = 0; i <= QMAX + 1; ++i) S.tau[i] = 0.0;
#pragma unroll
  for (int i = 0; i < 6; ++i) S.tq[i] = 0.0;
  S.hu = 0.0;
}

template <int N>
__device__ __forceinline__ int bdf_step(Bdf& b, BdfS& S, Wave<N>& w, int& nst_global) {
  const int n = w.n;
  const bool act = w.lane < n;
  const double saved_t = S.tn;
  int ncf = 0, nef = 0, nflag = NF_FIRST;
  double dsm;
  if (S.nst > 0 && S.hprime != S.h) {
    if (S.qprime != S.q) {
      bdf_adjust_order(b, S, S.qprime - S.q);
      S.q = S.qprime;
      S.L = S.q + 1;
      S.qwait = S.L;
    }
    bdf_rescale(b, S);
  }
  for (;;) {
    bdf_predict(b, S);
    bdf_set(b, S);
    const int r = bdf_nls<N>(b, S, w, nflag);
    if (r != 0) {
      ncf++;
      S.ncf_tot++;
      S.etamax = 1.0;
      bdf_restore(b, S, saved_t);
      if (fabs(S.h) <= S.hmin * ONEPSM || ncf == MXNCF) return CKMI_RUN_CONVFAIL;
      S.eta = fmax(ETACF, S.hmin / fabs(S.h));
      nflag = NF_CONV_FAIL;
      bdf_rescale(b, S);
      continue;
    }
    dsm = S.acnrm * S.tq[2];
    if (dsm <= 1.0) break;
    nef++;
    S.nef_tot++;
    nflag = NF_ERR_FAIL;
    bdf_restore(b, S, saved_t);
    if (fabs(S.h) <= S.hmin * ONEPSM || nef == MXNEF) return CKMI_RUN_ERRTEST;
    S.etamax = 1.0;
    if (nef <= MXNEF1) {
      S.eta = 1.0 / (pow(BIAS2 * dsm, 1.0 / S.L) + ADDON);
      S.eta = fmax(ETAMIN, fmax(S.eta, S.hmin / fabs(S.h)));
      if (nef >= SMALL_NEF) S.eta = fmin(S.eta, ETAMXF);
      bdf_rescale(b, S);
      continue;
    }
    if (S.q > 1) {
      S.eta = fmax(ETAMIN, S.hmin / fabs(S.h));
      bdf_adjust_order(b, S, -1);
      S.L = S.q;
      S.q--;
      S.qwait = S.L;
      bdf_rescale(b, S);
      continue;
    }
    S.eta = fmax(ETAMIN, S.hmin / fabs(S.h));
    S.h *= S.eta;
    S.hscale = S.h;
    S.qwait = LONG_WAIT;
    const double fz = w.f(S.tn, b.zn[0]);
    S.nfe++;
    b.zn[1] = act ? S.h * fz : 0.0;
  }
  // complete the step
  S.nst++;
  nst_global++;
  S.hu = S.h;
#pragma unroll
  for (int i = QMAX; i >= 2; --i)
    if (i <= S.q) S.tau[i] = S.tau[i - 1];
  if (S.q == 1 && S.nst > 1) S.tau[2] = S.tau[1];
  S.tau[1] = S.h;
#pragma unroll
  for (int j = 0; j <= QMAX; ++j)
    if (j <= S.q) b.zn[j] += S.l[j] * b.acor;
  S.qwait--;
  if (S.qwait == 1 && S.q != QMAX) {
    b.zn[QMAX] = b.acor;
    S.saved_tq5 = S.tq[5];
  }
  // prepare the next step
  if (S.etamax == 1.0) {
    if (S.qwait < 2) S.qwait = 2;
    S.qprime = S.q;
    S.hprime = S.h;
    S.eta = 1.0;
  } else {
    const double etaq = 1.0 / (pow(BIAS2 * dsm, 1.0 / S.L) + ADDON);
    if (S.qwait != 0) {
      S.eta = etaq;
      S.qprime = S.q;
    } else {
      S.qwait = 2;
      double etaqm1 = 0.0, etaqp1 = 0.0;
      if (S.q > 1) {
        double znq = 0.0;
#pragma unroll
        for (int j = 0; j <= QMAX; ++j)
          if (j == S.q) znq = b.zn[j];
        const double ddn = wrms_lane(act ? znq : 0.0, b.ewt, n) * S.tq[1];
        etaqm1 = 1.0 / (pow(BIAS1 * ddn, 1.0 / S.q) + ADDON);
      }
      if (S.q != QMAX && S.saved_tq5 != 0.0) {
        const double cquot = (S.tq[5] / S.saved_tq5) * pow(S.h / S.tau[2], (double)S.L);
        const double tv = act ? b.acor - cquot * b.zn[QMAX] : 0.0;
        const double dup = wrms_lane(tv, b.ewt, n) * S.tq[3];
        etaqp1 = 1.0 / (pow(BIAS3 * dup, 1.0 / (S.L + 1)) + ADDON);
      }
      const double etam = fmax(etaqm1, fmax(etaq, etaqp1));
      if (etam < THRESH) {
        S.eta = 1.0;
        S.qprime = S.q;
      } else if (etam == etaq) {
        S.eta = etaq;
        S.qprime = S.q;
      } else if (etam == etaqm1) {
        S.eta = etaqm1;
        S.qprime = S.q - 1;
      } else {
        S.eta = etaqp1;
        S.qprime = S.q + 1;
        b.zn[QMAX] = b.acor;
      }
    }
    if (S.eta < THRESH) {
      S.eta = 1.0;
      S.hprime = S.h;
    } else {
      S.eta = fmin(S.eta, S.etamax);
      S.eta /= fmax(1.0, fabs(S.h) * S.hmax_inv * S.eta);
      S.hprime = S.h * S.eta;
    }
  }
  S.etamax = (S.nst <= SMALL_NST) ? ETAMX2 : ETAMX3;
  return 0;
}

// ignition monitor (uniform scalars), mirrors oracle ign_* helpers
struct Ign {
  int mode, comp, found, started, have_prev, have_next;
  double thresh, best, tbest, tprev, vprev, tnext, vnext, tlast, vlast, tau;
};

__device__ __forceinline__ void ign_peak_update(Ign& g, double t, double v) {
  if (g.started && g.found == 0 && v > g.best) {
    g.tprev = g.tlast;
    g.vprev = g.vlast;
    g.have_prev = 1;
    g.best = v;
    g.tbest = t;
    g.have_next = 0;
  } else if (g.started && !g.have_next && g.tbest != 0.0 && t > g.tbest) {
    g.tnext = t;
    g.vnext = v;
    g.have_next = 1;
  } else if (!g.started) {
    g.best = v;
    g.tbest = t;
    g.have_prev = 0;
  }
  g.started = 1;
  g.tlast = t;
  g.vlast = v;
}

__device__ __forceinline__ double ign_peak_time(const Ign& g) {
  if (g.tbest <= 0.0) return -1.0;
  if (!(g.have_prev && g.have_next)) return g.tbest;
  const double x0 = g.tprev, x1 = g.tbest, x2 = g.tnext;
  const double y0 = g.vprev, y1 = g.best, y2 = g.vnext;
  const double d01 = (y1 - y0) / (x1 - x0), d12 = (y2 - y1) / (x2 - x1);
  const double a = (d12 - d01) / (x2 - x0);
  if (!(a < 0.0)) return x1;
  const double bc = d01 - a * (x0 + x1);
  const double tv = -bc / (2.0 * a);
  if (tv < x0 || tv > x2) return x1;
  return tv;
}

__device__ __forceinline__ int n_crit(const ckmi_reactor_cfg* c, double tend) {
  int k = 0;
  for (int i = 0; i < c->nprof; ++i)
    if (c->prof_t[i] > 0.0 && c->prof_t[i] < tend) ++k;
  return k + 1;
}
__device__ __forceinline__ double crit_time(const ckmi_reactor_cfg* c, double tend, int idx) {
  int k = 0;
  for (int i = 0; i < c->nprof; ++i)
    if (c->prof_t[i] > 0.0 && c->prof_t[i] < tend) {
      if (k == idx) return c->prof_t[i];
      ++k;
    }
  return tend;
}

__device__ __forceinline__ void state_PV(const MechDev& M, const RunCtx& R, double t, double yl, int lane, double& P,
                                         double& V) {
  const int KK = M.KK;
  const bool isp = lane >= 1 && lane <= KK;
  const double T = bcast(yl, 0);
  const double Wb = 1.0 / wave_sum(isp ? yl * M.rwt[lane - 1] : 0.0);
  double d;
  if (R.conp) {
    profile_eval(R.cfg, R.cfg->nprof, t, R.P0, P, d);
    const double rho = P * Wb / (RU * T);
    V = R.rho0 * R.V0 / rho;
  } else {
    profile_eval(R.cfg, R.cfg->nprof, t, R.V0, V, d);
    const double rho = R.rho0 * R.V0 / V;
    P = rho * RU * T / Wb;
  }
}

template <int N>
__global__ __launch_bounds__(WAVE) void reactor_kernel(MechDev M, const ckmi_reactor_cfg* __restrict__ cfg, int nreact,
                                                       const int* __restrict__ problem, const double* __restrict__ T0v,
                                                       const double* __restrict__ P0v, const double* __restrict__ V0v,
                                                       const double* __restrict__ Y0v, double* __restrict__ tau_o,
                                                       double* __restrict__ T_o, double* __restrict__ P_o,
                                                       double* __restrict__ V_o, double* __restrict__ Y_o,
                                                       int* __restrict__ stats_o, int nsave,
                                                       const double* __restrict__ t_save,
                                                       double* __restrict__ y_save) {
  extern __shared__ double lds[];
  const int r = blockIdx.x;
  if (r >= nreact) return;
  const int lane = threadIdx.x;
  const int KK = M.KK;
  const int n = KK + 1;
  const int ld = (n & 1) ? n : n + 1;
  const int VL = (KK + WAVE - 1) / WAVE * WAVE;
  Lds L;
  L.J = lds;
  L.A = L.J + ((n * ld + 1) & ~1);
  L.C = L.A + ((n * ld + 1) & ~1);
  L.gRT = L.C + VL;
  L.hRT = L.gRT + VL;
  L.wdot = L.hRT + VL;
  L.dwdT = L.wdot + VL;
  L.ek = L.dwdT + VL;
  L.Mg = L.ek + VL;

  const bool isp = lane >= 1 && lane <= KK;
  const bool act = lane < n;
  const int prob = problem[r];
  const double T0 = T0v[r], P0 = P0v[r];
  double yl = 0.0;
  if (lane == 0) yl = T0;
  if (isp) yl = Y0v[(size_t)r * KK + lane - 1];
  const double Wbar0 = 1.0 / wave_sum(isp ? yl * M.rwt[lane - 1] : 0.0);
  const double rho0 = P0 * Wbar0 / (RU * T0);
  RunCtx R;
  R.conp = (prob == 1);
  R.energy = cfg->energy;
  R.rho0 = rho0;
  R.cfg = cfg;
  R.V0 = (!R.conp && cfg->nprof > 0) ? cfg->prof_v[0] : V0v[r];
  R.P0 = (R.conp && cfg->nprof > 0) ? cfg->prof_v[0] : P0;

  Wave<N> w(M, R, L, lane, n, ld);
  __shared__ BdfS S;
  __shared__ Ign g;
  Bdf b;
  S.rtol = cfg->rtol;
  S.atol = cfg->atol;
  S.nneg = cfg->nneg;
  S.ncf_tot = S.nef_tot = S.nlu = S.nfe = S.nje = S.nni = 0;
  const double tend = cfg->t_end;
  const double hmax = cfg->hmax > 0.0 ? cfg->hmax : tend / 100.0;
  S.hmax_inv = 1.0 / hmax;
  S.hmin = 0.0;
  const int ncrit = n_crit(cfg, tend);
  int icrit = 0;
  bdf_start<N>(b, S, w, 0.0, yl, crit_time(cfg, tend, 0), cfg->h0, hmax);

  g.mode = cfg->ign_mode;
  g.comp = (g.mode == 4) ? 1 + cfg->ign_species : 0;
  g.found = g.started = g.have_prev = g.have_next = 0;
  g.thresh = 0.0;
  g.best = -1e300;
  g.tbest = g.tprev = g.vprev = g.tnext = g.vnext = g.tlast = g.vlast = 0.0;
  g.tau = -1.0;
  if (g.mode == 2) g.thresh = T0 + cfg->ign_val;
  if (g.mode == 3) g.thresh = cfg->ign_val;

  int isave = 0;
  while (isave < nsave && t_save[isave] <= 0.0) {
    if (act) y_save[((size_t)r * nsave + isave) * n + lane] = yl;
    isave++;
  }
  if (g.mode == 1 || g.mode == 4) {
    const double f0 = w.f(0.0, yl);
    S.nfe++;
    ign_peak_update(g, 0.0, g.mode == 1 ? bcast(f0, 0) : bcast(yl, g.comp));
  }
  int status = 0, nst = 0, stopped = 0;
  const int max_steps = cfg->max_steps > 0 ? cfg->max_steps : 200000;
  while (S.tn < tend * (1.0 - 1e-15)) {
    const double tc = crit_time(cfg, tend, icrit);
    if (S.tn + S.hprime > tc) {
      const double hp = tc - S.tn;
      S.eta = hp / S.h;
      if (S.nst > 0) {
        S.hprime = hp;
      } else {
        bdf_rescale(b, S);
        S.hprime = S.h;
      }
    }
    b.ewt = act ? 1.0 / (S.rtol * fabs(b.zn[0]) + S.atol) : 0.0;
    const double told = S.tn;
    const int rc = bdf_step<N>(b, S, w, nst);
    if (rc != 0) {
      status = rc;
      break;
    }
    const double tn = S.tn;
    while (isave < nsave && t_save[isave] <= tn) {
      const double ys = dky0_lane(b, S, t_save[isave]);
      if (act) y_save[((size_t)r * nsave + isave) * n + lane] = ys;
      isave++;
    }
    if (g.mode == 1) {
      ign_peak_update(g, tn, bcast(b.zn[1], 0) / S.h);
    } else if (g.mode == 4) {
      ign_peak_update(g, tn, bcast(b.zn[0], g.comp));
    } else if ((g.mode == 2 || g.mode == 3) && !g.found && bcast(b.zn[0], 0) >= g.thresh) {
      double lo = told, hi = tn;
      for (int it = 0; it < 60; ++it) {
        const double mid = 0.5 * (lo + hi);
        if (bcast(dky0_lane(b, S, mid), 0) >= g.thresh) hi = mid;
        else lo = mid;
      }
      g.found = 1;
      g.tau = hi;
    }
    if (cfg->ign_stop) {
      if ((g.mode == 2 || g.mode == 3) && g.found) {
        stopped = 1;
        break;
      }
      if (g.mode == 1 && g.have_next && g.vlast < 0.1 * g.best && bcast(b.zn[0], 0) > T0 + 200.0) {
        stopped = 1;
        break;
      }
    }
    if (nst >= max_steps) {
      status = CKMI_RUN_MAXSTEPS;
      break;
    }
    if (tn >= tc * (1.0 - 1e-15) && icrit < ncrit - 1) {
      const double yc = b.zn[0];
      icrit++;
      const int nlu = S.nlu, ncf = S.ncf_tot, nef = S.nef_tot;
      bdf_start<N>(b, S, w, tn, yc, crit_time(cfg, tend, icrit), 0.0, hmax);
      S.nlu = nlu;
      S.ncf_tot = ncf;
      S.nef_tot = nef;
    }
  }
  double yf;
  double tf = tend;
  if (stopped || status) {
    tf = S.tn;
    yf = b.zn[0];
  } else {
    yf = dky0_lane(b, S, tend);
  }
  if (g.mode == 1 || g.mode == 4) g.tau = ign_peak_time(g);
  double Pf, Vf;
  state_PV(M, R, tf, yf, lane, Pf, Vf);
  if (lane == 0) {
    tau_o[r] = g.tau;
    T_o[r] = yf;
    P_o[r] = Pf;
    V_o[r] = Vf;
    int* st = stats_o + (size_t)r * CKMI_NSTAT;
    st[CKMI_STAT_NST] = nst;
    st[CKMI_STAT_NFE] = S.nfe;
    st[CKMI_STAT_NJE] = S.nje;
    st[CKMI_STAT_NLU] = S.nlu;
    st[CKMI_STAT_NCF] = S.ncf_tot;
    st[CKMI_STAT_NEF] = S.nef_tot;
    st[CKMI_STAT_STATUS] = status;
    st[CKMI_STAT_NNI] = S.nni;
  }
  if (isp) Y_o[(size_t)r * KK + lane - 1] = yf;
}

// ---------------------------------------------------------------- ROP kernels
// One wave per state (lanes over reactions), SoA inputs [KK][n].
template <int MODE>  // 0: wdot + cp + h, 1: qf / qr
__global__ __launch_bounds__(WAVE) void rop_kernel(MechDev M, int nstate, const double* __restrict__ Tv,
                                                   const double* __restrict__ Pv, const double* __restrict__ Yv,
                                                   double* __restrict__ o0, double* __restrict__ o1,
                                                   double* __restrict__ o2) {
  extern __shared__ double lds[];
  const int st = blockIdx.x;
  if (st >= nstate) return;
  const int lane = threadIdx.x;
  const int KK = M.KK;
  const int VL = (KK + WAVE - 1) / WAVE * WAVE;
  double* C = lds;
  double* gRT = C + VL;
  double* wdot = gRT + VL;
  double* Mg = wdot + VL;
  const double T = Tv[st], P = Pv[st];
  double yk[2] = {0.0, 0.0};  // up to 128 species per state
  double rwv[2] = {0.0, 0.0};
  double s = 0.0;
#pragma unroll
  for (int c = 0; c < 2; ++c) {
    const int k = lane + c * WAVE;
    if (k < KK) {
      yk[c] = Yv[(size_t)k * nstate + st];
      rwv[c] = M.rwt[k];
      s += yk[c] * rwv[c];
    }
  }
  const double Wbar = 1.0 / wave_sum(s);
  const double rho = P * Wbar / (RU * T);
  const double lnT = log(T), invT = 1.0 / T, lnPRT = log(PATM / (RU * T));
  double cpm = 0.0, hm = 0.0, ctot = 0.0;
  for (int k = lane; k < KK; k += WAVE) {
    const int c = k / WAVE;
    const SpThermo th = nasa7(M, k, T, lnT);
    const double Ck = rho * yk[c] * rwv[c];
    C[k] = Ck;
    gRT[k] = th.hRT - th.sR;
    wdot[k] = 0.0;
    ctot += Ck;
    cpm += yk[c] * th.cpR * RU * rwv[c];
    hm += yk[c] * th.hRT * RU * T * rwv[c];
  }
  const double Ctot = wave_sum(ctot);
  __syncthreads();
  for (int g = lane; g < M.G; g += WAVE) {
    double m = Ctot;
    for (int p = M.gptr[g]; p < M.gptr[g + 1]; ++p) m += M.geff[p] * C[M.gsp[p]];
    Mg[g] = m;
  }
  __syncthreads();
  const int IIp = M.IIpad;
  for (int base = 0; base < IIp; base += WAVE) {
    const int i = base + lane;
    const int nrp = M.nrp[i];
    const int nr = nrp & 0xff, np = nrp >> 8;
    if (nr + np == 0) continue;
    const RxnEval e = eval_rxn(M, i, T, lnT, invT, lnPRT, C, gRT, nullptr, Mg, false);
    const double qf = e.mfac * e.kf * e.pf, qr = e.mfac * e.kr * e.pr;
    if (MODE == 1) {
      const int oi = M.orig[i];
      o0[(size_t)oi * nstate + st] = qf;
      o1[(size_t)oi * nstate + st] = qr;
    } else {
      const double q = qf - qr;
      const int4 rs = M.rsp[i], ps = M.psp[i];
#pragma unroll
      for (int u = 0; u < SLOTS; ++u) {
        if (u < nr) atomicAdd(&wdot[slot(rs, u)], -M.rnu[u * IIp + i] * q);
        if (u < np) atomicAdd(&wdot[slot(ps, u)], M.pnu[u * IIp + i] * q);
      }
    }
  }
  if (MODE == 0) {
    __syncthreads();
    for (int k = lane; k < KK; k += WAVE) o0[(size_t)k * nstate + st] = wdot[k];
    const double cps = wave_sum(cpm), hs = wave_sum(hm);
    if (lane == 0) {
      if (o1) o1[st] = cps;
      if (o2) o2[st] = hs;
    }
  }
}

// species thermo: one thread per state, coefficients read uniformly
__global__ void species_thermo_kernel(MechDev M, int nstate, const double* __restrict__ Tv, double* __restrict__ cp,
                                      double* __restrict__ h, double* __restrict__ s) {
  const int st = blockIdx.x * blockDim.x + threadIdx.x;
  if (st >= nstate) return;
  const double T = Tv[st], lnT = log(T);
  for (int k = 0; k < M.KK; ++k) {
    const SpThermo th = nasa7(M, k, T, lnT);
    if (cp) cp[(size_t)k * nstate + st] = th.cpR;
    if (h) h[(size_t)k * nstate + st] = th.hRT;
    if (s) s[(size_t)k * nstate + st] = th.sR;
  }
}

}  // namespace

// ====================================================================== host side
struct ckmi_mech {
  int device;
  int KK, II, IIpad, G;
  MechDev d;
  std::vector<void*> allocs;
  // host copies of the forward Arrhenius (original order) for get/set
  std::vector<double> lnA_orig, b_orig, E_orig;
  std::vector<int> slot_of;  // original reaction -> device slot
  ckmi_reactor_cfg* cfg_dev;
};

namespace {

template <typename T>
int upload(ckmi_mech* m, const std::vector<T>& v, const T** out) {
  void* p = nullptr;
  size_t bytes = std::max<size_t>(v.size() * sizeof(T), 16);
  HIP_CHECK(hipMalloc(&p, bytes));
  if (!v.empty()) HIP_CHECK(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
  m->allocs.push_back(p);
  *out = static_cast<const T*>(p);
  return CKMI_OK;
}

size_t reactor_lds_bytes(int KK, int G) {
  const int n = KK + 1;
  const int ld = (n & 1) ? n : n + 1;
  const int VL = (KK + WAVE - 1) / WAVE * WAVE;
  return sizeof(double) * (size_t)(2 * ((n * ld + 1) & ~1) + 6 * VL + std::max(G, 1));
}
size_t rop_lds_bytes(int KK, int G) {
  const int VL = (KK + WAVE - 1) / WAVE * WAVE;
  return sizeof(double) * (size_t)(3 * VL + std::max(G, 1));
}

}  // namespace

extern "C" {

const char* ckmi_last_error(void) { return g_err.c_str(); }
int ckmi_version(void) { return 1; }

int ckmi_mech_create(const ckmi_mech_desc* d, ckmi_mech** out) {
  if (!d || !out) return fail(CKMI_ERR_ARG, "null argument");
  const int KK = d->KK, II = d->II;
  if (KK <= 0 || II < 0) return fail(CKMI_ERR_SIZE, "bad sizes");
  if (KK + 1 > 64) return fail(CKMI_ERR_UNSUPPORTED, "more than 63 species not supported by this build");
  auto* m = new ckmi_mech();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    delete m;
    return fail(CKMI_ERR_HIP, "no HIP device");
  }
  m->device = dev;
  m->KK = KK;
  m->II = II;
  // ---- order reactions: elementary, then third-body, then falloff
  std::vector<int> ordr;
  for (int t = 0; t < 3; ++t)
    for (int i = 0; i < II; ++i)
      if (d->rtype[i] == t) ordr.push_back(i);
  for (int i = 0; i < II; ++i)
    if (d->rtype[i] < 0 || d->rtype[i] > 2) {
      delete m;
      return fail(CKMI_ERR_UNSUPPORTED, "unsupported reaction type");
    }
  // pad the elementary block to a 64 multiple when it does not add a strip
  int nelem = 0;
  for (int i = 0; i < II; ++i) nelem += d->rtype[i] == 0;
  std::vector<int> slots;  // device slot -> original index (-1 pad)
  const int strips_nopad = (II + WAVE - 1) / WAVE;
  const int elem_pad = (nelem + WAVE - 1) / WAVE * WAVE;
  const int strips_pad = (elem_pad + (II - nelem) + WAVE - 1) / WAVE;
  const bool pad = nelem > 0 && nelem < II && strips_pad == strips_nopad;
  for (int s = 0; s < (int)ordr.size(); ++s) {
    if (pad && s == nelem)
      while ((int)slots.size() < elem_pad) slots.push_back(-1);
    slots.push_back(ordr[s]);
  }
  const int IIpad = std::max(WAVE, (int)((slots.size() + WAVE - 1) / WAVE * WAVE));
  while ((int)slots.size() < IIpad) slots.push_back(-1);
  m->IIpad = IIpad;
  m->slot_of.assign(II, -1);
  // ---- third-body groups (distinct efficiency lists)
  std::map<std::vector<std::pair<int, double>>, int> gmap;
  std::vector<int> gptr{0}, gsp;
  std::vector<double> geff;
  auto group_of = [&](int i) -> int {
    std::vector<std::pair<int, double>> key;
    for (int p = d->eff_ptr[i]; p < d->eff_ptr[i + 1]; ++p)
      if (d->eff_val[p] != 1.0) key.push_back({d->eff_sp[p], d->eff_val[p] - 1.0});
    std::sort(key.begin(), key.end());
    auto it = gmap.find(key);
    if (it != gmap.end()) return it->second;
    const int gid = (int)gmap.size();
    gmap[key] = gid;
    for (auto& kv : key) {
      gsp.push_back(kv.first);
      geff.push_back(kv.second);
    }
    gptr.push_back((int)gsp.size());
    return gid;
  };
  std::vector<int> flags(IIpad, 0), nrp(IIpad, 0), tb(IIpad, -1), orig(IIpad, -1);
  std::vector<int4> rsp(IIpad), psp(IIpad);
  std::vector<double> rnu(SLOTS * IIpad, 0.0), pnu(SLOTS * IIpad, 0.0);
  std::vector<double> lnA(IIpad, 0.0), beta(IIpad, 0.0), Ea(IIpad, 0.0), lnA0(IIpad, 0.0), beta0(IIpad, 0.0),
      Ea0(IIpad, 0.0), fp(5 * IIpad, 1.0), rlnA(IIpad, 0.0), rbeta(IIpad, 0.0), rEa(IIpad, 0.0), dnu(IIpad, 0.0),
      ordf(IIpad, 0.0), ordrr(IIpad, 0.0);
  for (int s = 0; s < IIpad; ++s) {
    rsp[s] = make_int4(0, 0, 0, 0);
    psp[s] = make_int4(0, 0, 0, 0);
    const int i = slots[s];
    orig[s] = i;
    if (i < 0) continue;
    m->slot_of[i] = s;
    const int type = d->rtype[i];
    flags[s] = type | (d->rev[i] ? 4 : 0) | (d->has_rev[i] ? 8 : 0) | ((d->ftype[i] & 7) << 4);
    const int nr = d->nr[i], np = d->np[i];
    for (int u = 0; u < nr; ++u)
      if (d->rnu[i * SLOTS + u] != std::floor(d->rnu[i * SLOTS + u]) || d->rnu[i * SLOTS + u] < 1.0) {
        delete m;
        return fail(CKMI_ERR_UNSUPPORTED, "non-integral stoichiometric coefficient");
      }
    for (int u = 0; u < np; ++u)
      if (d->pnu[i * SLOTS + u] != std::floor(d->pnu[i * SLOTS + u]) || d->pnu[i * SLOTS + u] < 1.0) {
        delete m;
        return fail(CKMI_ERR_UNSUPPORTED, "non-integral stoichiometric coefficient");
      }
    if (nr > SLOTS || np > SLOTS) {
      delete m;
      return fail(CKMI_ERR_UNSUPPORTED, "more than 4 species on a reaction side");
    }
    nrp[s] = nr | (np << 8);
    int rr[4] = {0, 0, 0, 0}, pp[4] = {0, 0, 0, 0};
    double sf = 0.0, sr = 0.0;
    for (int u = 0; u < nr; ++u) {
      rr[u] = d->rsp[i * SLOTS + u];
      rnu[u * IIpad + s] = d->rnu[i * SLOTS + u];
      sf += d->rnu[i * SLOTS + u];
    }
    for (int u = 0; u < np; ++u) {
      pp[u] = d->psp[i * SLOTS + u];
      pnu[u * IIpad + s] = d->pnu[i * SLOTS + u];
      sr += d->pnu[i * SLOTS + u];
    }
    rsp[s] = make_int4(rr[0], rr[1], rr[2], rr[3]);
    psp[s] = make_int4(pp[0], pp[1], pp[2], pp[3]);
    dnu[s] = sr - sf;
    ordf[s] = sf;
    ordrr[s] = sr;
    lnA[s] = d->arr[3 * i];
    beta[s] = d->arr[3 * i + 1];
    Ea[s] = d->arr[3 * i + 2];
    lnA0[s] = d->low[3 * i];
    beta0[s] = d->low[3 * i + 1];
    Ea0[s] = d->low[3 * i + 2];
    for (int c = 0; c < 5; ++c) fp[c * IIpad + s] = d->fpar[5 * i + c];
    rlnA[s] = d->revp[3 * i];
    rbeta[s] = d->revp[3 * i + 1];
    rEa[s] = d->revp[3 * i + 2];
    if (type != 0) tb[s] = d->tbsp[i] >= 0 ? -(d->tbsp[i] + 2) : group_of(i);
  }
  m->G = (int)gmap.size();
  m->lnA_orig.resize(II);
  m->b_orig.resize(II);
  m->E_orig.resize(II);
  for (int i = 0; i < II; ++i) {
    m->lnA_orig[i] = d->arr[3 * i];
    m->b_orig[i] = d->arr[3 * i + 1];
    m->E_orig[i] = d->arr[3 * i + 2];
  }
  std::vector<double> wt(d->wt, d->wt + KK), rwt(KK), th(17 * KK);
  for (int k = 0; k < KK; ++k) {
    rwt[k] = 1.0 / wt[k];
    for (int c = 0; c < 17; ++c) th[c * KK + k] = d->thermo[17 * k + c];
  }
  MechDev& D = m->d;
  D.KK = KK;
  D.II = II;
  D.IIpad = IIpad;
  D.G = m->G;
  int rc = 0;
  rc |= upload(m, wt, &D.wt);
  rc |= upload(m, rwt, &D.rwt);
  rc |= upload(m, th, &D.th);
  rc |= upload(m, flags, &D.flags);
  rc |= upload(m, nrp, &D.nrp);
  rc |= upload(m, rsp, &D.rsp);
  rc |= upload(m, psp, &D.psp);
  rc |= upload(m, rnu, &D.rnu);
  rc |= upload(m, pnu, &D.pnu);
  rc |= upload(m, lnA, &D.lnA);
  rc |= upload(m, beta, &D.beta);
  rc |= upload(m, Ea, &D.Ea);
  rc |= upload(m, lnA0, &D.lnA0);
  rc |= upload(m, beta0, &D.beta0);
  rc |= upload(m, Ea0, &D.Ea0);
  rc |= upload(m, fp, &D.fp);
  rc |= upload(m, rlnA, &D.rlnA);
  rc |= upload(m, rbeta, &D.rbeta);
  rc |= upload(m, rEa, &D.rEa);
  rc |= upload(m, dnu, &D.dnu);
  rc |= upload(m, ordf, &D.ordf);
  rc |= upload(m, ordrr, &D.ordr);
  rc |= upload(m, tb, &D.tb);
  rc |= upload(m, orig, &D.orig);
  rc |= upload(m, gptr, &D.gptr);
  rc |= upload(m, gsp, &D.gsp);
  rc |= upload(m, geff, &D.geff);
  void* cp = nullptr;
  if (hipMalloc(&cp, sizeof(ckmi_reactor_cfg)) != hipSuccess) rc |= CKMI_ERR_HIP;
  else m->allocs.push_back(cp);
  m->cfg_dev = static_cast<ckmi_reactor_cfg*>(cp);
  if (rc) {
    ckmi_mech_destroy(m);
    return rc;
  }
  *out = m;
  return CKMI_OK;
}

int ckmi_mech_destroy(ckmi_mech* m) {
  if (!m) return CKMI_OK;
  for (void* p : m->allocs) (void)hipFree(p);
  delete m;
  return CKMI_OK;
}

int ckmi_mech_sizes(const ckmi_mech* m, int32_t* KK, int32_t* II) {
  if (!m) return fail(CKMI_ERR_ARG, "null mech");
  if (KK) *KK = m->KK;
  if (II) *II = m->II;
  return CKMI_OK;
}

int ckmi_get_arrhenius(const ckmi_mech* m, double* A, double* b, double* E) {
  if (!m) return fail(CKMI_ERR_ARG, "null mech");
  for (int i = 0; i < m->II; ++i) {
    if (A) A[i] = std::exp(m->lnA_orig[i]);
    if (b) b[i] = m->b_orig[i];
    if (E) E[i] = m->E_orig[i];
  }
  return CKMI_OK;
}

int ckmi_set_afactor(ckmi_mech* m, int32_t irxn, double A) {
  if (!m || irxn < 0 || irxn >= m->II || !(A > 0.0)) return fail(CKMI_ERR_ARG, "bad reaction index or A");
  const double lnA = std::log(A);
  m->lnA_orig[irxn] = lnA;
  const int s = m->slot_of[irxn];
  HIP_CHECK(hipMemcpy(const_cast<double*>(m->d.lnA) + s, &lnA, sizeof(double), hipMemcpyHostToDevice));
  return CKMI_OK;
}

int ckmi_species_thermo(const ckmi_mech* m, int32_t n, const double* T, double* cp_R, double* h_RT, double* s_R,
                        void* stream) {
  if (!m || n < 0) return fail(CKMI_ERR_ARG, "bad argument");
  if (n == 0) return CKMI_OK;
  const int bs = 256;
  hipLaunchKernelGGL(species_thermo_kernel, dim3((n + bs - 1) / bs), dim3(bs), 0, (hipStream_t)stream, m->d, n, T, cp_R,
                     h_RT, s_R);
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

int ckmi_rop_thermo(const ckmi_mech* m, int32_t n, const double* T, const double* P, const double* Y, double* wdot,
                    double* cp, double* h, void* stream) {
  if (!m || n < 0 || !wdot) return fail(CKMI_ERR_ARG, "bad argument");
  if (n == 0) return CKMI_OK;
  hipLaunchKernelGGL(rop_kernel<0>, dim3(n), dim3(WAVE), rop_lds_bytes(m->KK, m->G), (hipStream_t)stream, m->d, n, T, P,
                     Y, wdot, cp, h);
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

int ckmi_reaction_rates(const ckmi_mech* m, int32_t n, const double* T, const double* P, const double* Y, double* qf,
                        double* qr, void* stream) {
  if (!m || n < 0 || !qf || !qr) return fail(CKMI_ERR_ARG, "bad argument");
  if (n == 0) return CKMI_OK;
  hipLaunchKernelGGL(rop_kernel<1>, dim3(n), dim3(WAVE), rop_lds_bytes(m->KK, m->G), (hipStream_t)stream, m->d, n, T, P,
                     Y, qf, qr, (double*)nullptr);
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

int ckmi_reactor_run(const ckmi_mech* m, const ckmi_reactor_cfg* cfg, int32_t n, const int32_t* problem,
                     const double* T0, const double* P0, const double* V0, const double* Y0, double* tau, double* Tend,
                     double* Pend, double* Vend, double* Yend, int32_t* stats, int32_t nsave, const double* t_save,
                     double* y_save, void* stream) {
  if (!m || !cfg || n < 0) return fail(CKMI_ERR_ARG, "bad argument");
  if (cfg->nprof < 0 || cfg->nprof > 64) return fail(CKMI_ERR_ARG, "nprof must be in [0, 64]");
  if (!(cfg->t_end > 0.0) || !(cfg->rtol > 0.0) || !(cfg->atol > 0.0)) return fail(CKMI_ERR_ARG, "t_end, rtol, atol must be > 0");
  if (cfg->energy != 1 && cfg->energy != 2) return fail(CKMI_ERR_ARG, "energy must be 1 or 2");
  if (cfg->ign_mode < 0 || cfg->ign_mode > 4) return fail(CKMI_ERR_ARG, "bad ignition mode");
  if (cfg->ign_mode == 4 && (cfg->ign_species < 0 || cfg->ign_species >= m->KK)) return fail(CKMI_ERR_ARG, "bad KLIM species");
  if (nsave > 0 && (!t_save || !y_save)) return fail(CKMI_ERR_ARG, "t_save / y_save required when nsave > 0");
  if (n == 0) return CKMI_OK;
  HIP_CHECK(hipMemcpyAsync(m->cfg_dev, cfg, sizeof(ckmi_reactor_cfg), hipMemcpyHostToDevice, (hipStream_t)stream));
  const size_t lds = reactor_lds_bytes(m->KK, m->G);
  const int nvar = m->KK + 1;
  if (nvar <= 32) {
    hipLaunchKernelGGL(reactor_kernel<32>, dim3(n), dim3(WAVE), lds, (hipStream_t)stream, m->d, m->cfg_dev, n, problem, T0,
                       P0, V0, Y0, tau, Tend, Pend, Vend, Yend, stats, nsave, t_save, y_save);
  } else if (nvar <= 54) {
    hipLaunchKernelGGL(reactor_kernel<54>, dim3(n), dim3(WAVE), lds, (hipStream_t)stream, m->d, m->cfg_dev, n, problem, T0,
                       P0, V0, Y0, tau, Tend, Pend, Vend, Yend, stats, nsave, t_save, y_save);
  } else {
    hipLaunchKernelGGL(reactor_kernel<64>, dim3(n), dim3(WAVE), lds, (hipStream_t)stream, m->d, m->cfg_dev, n, problem, T0,
                       P0, V0, Y0, tau, Tend, Pend, Vend, Yend, stats, nsave, t_save, y_save);
  }
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

}  // extern "C"
