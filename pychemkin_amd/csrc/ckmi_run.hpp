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
  // element projection of the accepted corrector (oracle elem_project): elements in the image's element
  // table (0 = off: no element counts, more than CKMI_PROJ_MMAX elements, or cfg.no_elem_proj)
  int npe;
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
  double eb0[PROJ_MMAX];  // the reactor's initial element contents (element projection)
  double tdh;             // h dT/dt of the accepted state (workgroup kernel: from the step's fused reduction)
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
