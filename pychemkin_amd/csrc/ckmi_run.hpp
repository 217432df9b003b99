// ckmi_run.hpp -- run-level types shared by the reactor kernels (ckmi.hip: one wave per reactor,
// KK <= 63; ckmi_big.hip: one workgroup per reactor, 64 <= KK + 1 <= 192).
#pragma once
#include "ckmi_reactor.hpp"

namespace ckmi {

enum { NF_FIRST = 0, NF_CONV_FAIL = 1, NF_ERR_FAIL = 2 };
enum { CF_NONE = 0, CF_BAD_J = 1, CF_OTHER = 2 };

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

// Device copy of the run configuration: the public struct plus the integration stop points
// (the sorted union of both profiles' breakpoints in (0, t_end), where derivatives jump),
// computed on the host by ckmi_reactor_run_ex.
struct DevCfg {
  ckmi_reactor_cfg c;
  int ncrit;
  double tcrit[192];  // breakpoints of the three profiles (64 each)
  // runaway guard (CKMI_RUN_RUNAWAY): -Y_k above guard_y, or T outside [guard_tlo, guard_thi]
  double guard_y, guard_tlo, guard_thi;
};
// true when an accepted state has left the physical domain (tested once per step by both kernels;
// oracle/ckoracle.c runaway() is the same test)
__device__ __forceinline__ bool runaway_value_bad(const DevCfg* d, double T) {
  return !(T >= d->guard_tlo && T <= d->guard_thi);
}
__device__ __forceinline__ int n_crit(const DevCfg* d) { return d->ncrit + 1; }
__device__ __forceinline__ double crit_time(const DevCfg* d, double tend, int idx) {
  return idx < d->ncrit ? d->tcrit[idx] : tend;
}

struct ReactorIO {
  const int* problem;
  const double *T0, *P0, *V0, *Y0;
  double *tau, *T, *P, *V, *Y;
  int* stats;
  int nsave;
  const double* t_save;
  double* y_save;
  // ckmi_reactor_ext
  const int* afac_rxn;
  const double* afac;
  int max_adap;
  double* t_adap;
  double* y_adap;
  int* n_adap;
  double* t_stop;
};

// Integrator control state of one wave (wave-uniform scalars, kept in the wave's LDS slice).
struct Ctl {
  int r, first, nflag, convfail, call_setup, failed, mm, ncf, nef, rc, isave, icrit, ncrit, status, nst, stopped;
  int is_count, max_steps, nadap;
  double avar_last;
  double delp, saved_t, told, dsm, tc, tend, hmax, T0;
  double yguard, tguard_lo, tguard_hi;  // runaway guard (DevCfg), copied per reactor
  double st_h0, st_tout, st_h, is_hg, is_hub, is_hlb, is_t0;
};

// ------------------------------------------------------------------ lane-resident integrator scalars
// The wave kernel keeps the integrator's wave-uniform scalars (BdfS and Ctl: 56 doubles, 34 ints) in
// one double and one int VGPR per lane, field j in lane j: reading a field is a v_readlane into an
// SGPR (a few cycles, usable as an operand at once), writing one a lane-select.  In LDS (round 1-3)
// every read was a ds_read round trip behind the strip gathers and atomics of 11 other waves: the
// bookkeeping between RHS calls took a third of a step.  The proxies below keep the member syntax of
// BdfS / Ctl (S.h, S.l[i], c.mm++ ...), so the shared BDF helpers compile for either storage.
struct LaneFile {
  double d;  // lane j: double field j
  int i;     // lane j: int field j
  int lane;  // this lane's index
};
__device__ __forceinline__ double lf_get(double r, int j) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(r), j);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(r), j);
  return __hiloint2double(hi, lo);
}
// write field j: the uniform value x into lane j (one compare, two selects)
__device__ __forceinline__ double lf_set(double r, int lane, int j, double x) { return lane == j ? uni(x) : r; }
struct PD {  // double field proxy
  LaneFile& f;
  int j;
  __device__ __forceinline__ operator double() const { return lf_get(f.d, j); }
  __device__ __forceinline__ PD& operator=(double x) {
    f.d = lf_set(f.d, f.lane, j, x);
    return *this;
  }
  __device__ __forceinline__ PD& operator=(const PD& o) { return *this = (double)o; }
  __device__ __forceinline__ PD& operator+=(double x) { return *this = (double)*this + x; }
  __device__ __forceinline__ PD& operator-=(double x) { return *this = (double)*this - x; }
  __device__ __forceinline__ PD& operator*=(double x) { return *this = (double)*this * x; }
  __device__ __forceinline__ PD& operator/=(double x) { return *this = (double)*this / x; }
};
struct PI {  // int field proxy
  LaneFile& f;
  int j;
  __device__ __forceinline__ operator int() const { return __builtin_amdgcn_readlane(f.i, j); }
  __device__ __forceinline__ PI& operator=(int x) {
    f.i = f.lane == j ? __builtin_amdgcn_readfirstlane(x) : f.i;
    return *this;
  }
  __device__ __forceinline__ PI& operator=(const PI& o) { return *this = (int)o; }
  __device__ __forceinline__ PI& operator+=(int x) { return *this = (int)*this + x; }
  __device__ __forceinline__ PI& operator-=(int x) { return *this = (int)*this - x; }
  __device__ __forceinline__ PI& operator++() { return *this += 1; }
  __device__ __forceinline__ int operator++(int) {
    const int v = *this;
    *this = v + 1;
    return v;
  }
  __device__ __forceinline__ PI& operator--() { return *this -= 1; }
  __device__ __forceinline__ int operator--(int) {
    const int v = *this;
    *this = v - 1;
    return v;
  }
};
template <int B>
struct PDA {  // double array field at lanes B, B + 1, ...
  LaneFile& f;
  __device__ __forceinline__ PD operator[](int k) const { return PD{f, B + k}; }
};
// BdfS over the lane file (same member names)
struct BdfR {
  LaneFile& f;
  PD h{f, 0}, hscale{f, 1}, hprime{f, 2}, eta{f, 3}, etamax{f, 4}, hmax_inv{f, 5}, hmin{f, 6}, tn{f, 7}, rl1{f, 8},
      gamma{f, 9}, gammap{f, 10}, gamrat{f, 11}, crate{f, 12}, acnrm{f, 13}, saved_tq5{f, 14}, hu{f, 15};
  PDA<16> l{f};   // [QMAX + 1]
  PDA<22> tq{f};  // [6]
  PDA<28> tau{f}; // [QMAX + 2]
  PD rtol{f, 35}, atol{f, 36};
  PI q{f, 0}, qprime{f, 1}, qwait{f, 2}, L{f, 3}, nst{f, 4}, nstlp{f, 5}, nstlj{f, 6}, jcur{f, 7}, ncf_tot{f, 8},
      nef_tot{f, 9}, nlu{f, 10}, nfe{f, 11}, nje{f, 12}, nni{f, 13}, nneg{f, 14};
  __device__ explicit BdfR(LaneFile& lf) : f(lf) {}
};
// Ctl over the lane file (same member names)
struct CtlR {
  LaneFile& f;
  PI r{f, 15}, first{f, 16}, nflag{f, 17}, convfail{f, 18}, call_setup{f, 19}, failed{f, 20}, mm{f, 21}, ncf{f, 22},
      nef{f, 23}, rc{f, 24}, isave{f, 25}, icrit{f, 26}, ncrit{f, 27}, status{f, 28}, nst{f, 29}, stopped{f, 30},
      is_count{f, 31}, max_steps{f, 32}, nadap{f, 33};
  PD avar_last{f, 37}, delp{f, 38}, saved_t{f, 39}, told{f, 40}, dsm{f, 41}, tc{f, 42}, tend{f, 43}, hmax{f, 44},
      T0{f, 45}, yguard{f, 46}, tguard_lo{f, 47}, tguard_hi{f, 48}, st_h0{f, 49}, st_tout{f, 50}, st_h{f, 51},
      is_hg{f, 52}, is_hub{f, 53}, is_hlb{f, 54}, is_t0{f, 55};
  __device__ explicit CtlR(LaneFile& lf) : f(lf) {}
};

// Per-wave LDS slice: 6 species vectors, third-body sums, integrator scalars, control state,
// ignition monitor.
__host__ __device__ constexpr int align16(int b) { return (b + 15) & ~15; }

// integrator states; the ones marked (f) resume after the RHS requested by their predecessor
enum {
  ST_NEXT = 0,       // pull the next reactor
  ST_START_F,        // (f) f(t, y0) for the Nordsieck history
  ST_INITSTEP_F,     // (f) one probe of the initial step-size estimate
  ST_START_FINISH,   // initial step chosen: set up the history
  ST_IGN0_F,         // (f) dT/dt at t = 0 for the inflection-point monitor
  ST_STEP_BEGIN,     // top of the time loop
  ST_STEP_ATTEMPT,   // predict + coefficients, begin a Newton solve
  ST_NLS_ATTEMPT,    // request f at the predictor
  ST_NLS_F,          // (f) f at the predictor; decide the Newton-matrix setup
  ST_NLS_J,          // (f) fresh Jacobian is in the shared scratch
  ST_SETUP,          // M = I - gamma J, LU
  ST_NEWTON_ITER,    // one Newton iteration
  ST_NEWTON_F,       // (f) f at the Newton iterate
  ST_NLS_FAIL,       // Newton failure: retry with a fresh J or fail the step
  ST_STEP_CONVFAIL,  // step failed to converge: shrink h
  ST_ERRTEST,        // local error test
  ST_ERR_F,          // (f) f after repeated error-test failures at order 1
  ST_STEP_COMPLETE,  // accept the step, choose the next h and q
  ST_STEP_END,       // outputs, ignition monitor, stops, critical-time restarts
  ST_FINISH,         // write the reactor's results
  ST_EXIT
};

}  // namespace ckmi
