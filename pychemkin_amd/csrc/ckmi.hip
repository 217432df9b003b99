// ckmi.hip -- gfx950 kernels and the C ABI of libckmi.so (see include/ckmi.h).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <vector>

#include "../../include/ckmi.h"
#include "ckmi_reactor.hpp"
#include "ckmi_run.hpp"
#include "ckmi_internal.hpp"

using namespace ckmi;

namespace {

thread_local std::string g_err;
// Kernel-path overrides (ckmi_set_reactor_path / ckmi_set_rop_path): process-wide test and A/B
// knobs, not per thread or per stream; each launch reads its selector once.
std::atomic<int> g_reactor_path{0};
std::atomic<int> g_rop_path{0};
constexpr int JIT_MIN_STATES = 16384;  // automatic choice: the specialised kernel from this batch size up

int fail(int code, const std::string& msg) {
  g_err = msg;
  return code;
}

#define HIP_CHECK(x)                                                                   \
  do {                                                                                 \
    hipError_t _e = (x);                                                               \
    if (_e != hipSuccess) return fail(CKMI_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)


// Diagnostic build only (-DCKMI_PHASE_TIMERS, scripts/phase_profile.py): per-reactor shader
// cycles spent in each phase, written to a debug buffer no other code reads.
// Slots 8..31 accumulate the cycles spent in each integrator state (RHS, LU, solve excluded).
enum { PH_RHS = 0, PH_JAC = 1, PH_LU = 2, PH_SOLVE = 3, PH_TOTAL = 4, PH_STATE = 8, PH_N = 48 };
#ifdef CKMI_PHASE_TIMERS
__device__ unsigned long long* g_phase_buf = nullptr;
#define PH_T0() const unsigned long long _ph0 = __builtin_amdgcn_s_memtime()
#define PH_ADD(slot) ph[slot] += __builtin_amdgcn_s_memtime() - _ph0
#else
#define PH_T0() (void)0
#define PH_ADD(slot) (void)0
#endif

// ---------------------------------------------------------------- reactor kernel
template <bool PF>
__device__ __forceinline__ void state_PV(const MechView& M, const RunCtx& R, double t, double yl, int lane, double& P,
                                         double& V) {
  const int KK = M.KK;
  const bool isp = lane >= 1 && lane <= KK;
  const double T = bcast(yl, 0);
  const double Wb = 1.0 / wave_sum(isp ? yl * M.rwt()[lane - 1] : 0.0);
  double d;
  if (PF && R.pfr == 2) {
    engine_volume(R.cfg->eng, t, V, d);
    P = (R.rho0 * R.V0 / V) * RU * T / Wb;
  } else if (PF && R.pfr == 1) {
    P = pfr_pressure(R.cfg, R.npv, R.G, R.Pm, t, t, T, Wb, d);
    V = R.G / (P * Wb / (RU * T));  // velocity
  } else if (R.conp) {
    profile_eval(R.cfg, R.npv, t, t, R.P0, P, d);
    const double rho = P * Wb / (RU * T);
    V = R.rho0 * R.V0 / rho;
  } else {
    profile_eval(R.cfg, R.npv, t, t, R.V0, V, d);
    const double rho = R.rho0 * R.V0 / V;
    P = rho * RU * T / Wb;
  }
}

__host__ __device__ constexpr int slice_vec_bytes(int G) { return align16(8 * (6 * VL + (G > 0 ? G : 1))); }
#ifdef CKMI_PHASE_TIMERS
constexpr int PH_SLICE = 8 * 40;  // per-state (0..19) and per-strip (24..29) cycle counters
#else
constexpr int PH_SLICE = 0;
#endif
__host__ __device__ constexpr int slice_bytes(int G) {
  return slice_vec_bytes(G) + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) + align16((int)sizeof(Ign)) +
         align16((int)sizeof(RunCtx)) + ZN_BYTES + PH_SLICE;
}
template <int N>
__host__ __device__ constexpr int jscratch_bytes() {
  return align16(8 * N * LDJ) + 16;  // + lock
}


// Persistent reactor kernel: one workgroup of RWAVES waves per CU slot.  The workgroup stages
// the mechanism image into LDS once; each wave then pulls reactor indices from an HBM work
// counter until the batch is exhausted (dynamic balancing: step counts differ by 10x across a
// T0 / phi / P sweep).  No workgroup barrier after staging, so waves run independently.
//
// The integrator (CVODE-style variable-order BDF with modified Newton, control flow identical
// to oracle/ckoracle.c) is written as a wave-uniform state machine whose only RHS evaluation,
// factorisation and solve each appear ONCE in the loop: the explicit inverse of M = I - gamma J
// then stays in VGPRs for the life of the wave.
// Waves per workgroup by Newton-matrix form: 12 (3 per SIMD) with the FP32-stored inverse, whose
// 54 VGPRs leave room for a third wave per SIMD within 168 VGPRs (+16 % reactors/s on configs[2]
// over 8 waves with the FP64 inverse, MI355X, although the 168-VGPR allocation spills ~28 values
// per step to scratch); 8 (2 per SIMD) with the FP64 inverse (256 VGPRs).
__host__ __device__ constexpr int rwaves(bool f64) { return f64 ? 8 : 12; }
// PL: the mechanism has PLOG / chemically activated / general reactions; F64: FP64-stored inverse.
// Plug flow (problem 3) is compiled into the FP64-inverse variants only (PF = F64): its branches
// cost the FP32-inverse variant, the configs[2] kernel, 12 B of scratch per lane and 0.5 % of its
// rate.  sel: 0 integrate every reactor, 1 skip the plug-flow reactors, 2 only those (the host
// pairs a sel 1 launch of an FP32-inverse variant with a sel 2 launch of an FP64 one).
enum { SEL_ALL = 0, SEL_NO_PFR = 1, SEL_PFR = 2 };
template <int N, bool PL = false, bool F64 = false>
__global__ __launch_bounds__(rwaves(F64)* WAVE) void reactor_kernel(MechImage img, const DevCfg* __restrict__ dcfg,
                                                               int nreact, int sel, int* __restrict__ queue,
                                                               double* __restrict__ jws, ReactorIO io) {
  constexpr bool PF = F64;
  const ckmi_reactor_cfg* __restrict__ cfg = &dcfg->c;
  const int oJ = img.bytes;
  const int olock = oJ + align16(8 * N * LDJ);
  if (threadIdx.x == 0) *lds_at<int>(olock) = 0;
  stage_image(0, img);
  const MechView V = make_view(0, img);
  const int wid = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int ows = oJ + jscratch_bytes<N>() + wid * slice_bytes(img.G);
  WaveLds L;
  L.base = ows;
  const int oS = ows + slice_vec_bytes(img.G);
  BdfS& S = *lds_at<BdfS>(oS);
  Ctl& c = *lds_at<Ctl>(oS + align16((int)sizeof(BdfS)));
  Ign& g = *lds_at<Ign>(oS + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)));
  // the wave's parked Jacobian, rounded to FP32: M = I - gamma J is rebuilt from it at every
  // setup (5.6 per J); the modified Newton iteration only needs an approximate M, and half
  // the bytes keep the slots of an XCD's 256 waves (3.5 MB) within its 4 MB L2
  constexpr int RWAVES = rwaves(F64);
  float* Jg = reinterpret_cast<float*>(jws) + ((size_t)blockIdx.x * RWAVES + wid) * N * WAVE;
  const int KK = V.KK;
  const int n = KK + 1;
  const bool isp = lane >= 1 && lane <= KK;
  const bool act = lane < n;
  // per-reactor constants of the RHS: in LDS, not registers (the Newton matrix owns those)
  RunCtx& R = *lds_at<RunCtx>(oS + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) + align16((int)sizeof(Ign)));
  R.cfg = cfg;
  std::conditional_t<F64, NewtonMatrixGJ64<N>, NewtonMatrixF32S<N>> M;
  Bdf b;
  b.zn.base = oS + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) + align16((int)sizeof(Ign)) +
              align16((int)sizeof(RunCtx)) + lane * 8;
  double fe = 0.0, y_e = 0.0, t_e = 0.0;
  bool with_j = false;
#ifdef CKMI_PHASE_TIMERS
  unsigned long long ph[8] = {0, 0, 0, 0, 0, 0, 0, 0};
  unsigned long long t_r0 = 0;
  unsigned long long* phs = lds_at<unsigned long long>(oS + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) +
                                                     align16((int)sizeof(Ign)) + align16((int)sizeof(RunCtx)) +
                                                     ZN_BYTES);
#endif
  int st = ST_NEXT;

  // request f at (t, y): sets the evaluation point and the state that consumes it
#define REQUEST_F(T_, Y_, NEXT_) \
  do {                           \
    t_e = (T_);                  \
    y_e = (Y_);                  \
    with_j = false;              \
    st = (NEXT_);                \
    want = true;                 \
  } while (0)
  // bdf_start: history at (t, y), then the initial step size (oracle bdf_start)
#define START_BEGIN(T_, Y_, TOUT_, H0_)                                 \
  do {                                                                 \
    S.tn = (T_);                                                       \
    b.zn[0] = act ? (Y_) : 0.0;                                        \
    _Pragma("unroll") for (int j_ = 1; j_ <= QMAX; ++j_) b.zn[j_] = 0.0; \
    b.ewt = act ? 1.0 / (S.rtol * fabs(b.zn[0]) + S.atol) : 0.0;       \
    c.st_tout = (TOUT_);                                               \
    R.tsel = 0.5 * (S.tn + c.st_tout);                                 \
    c.st_h0 = (H0_);                                                   \
    REQUEST_F(S.tn, b.zn[0], ST_START_F);                              \
  } while (0)

  for (;;) {
    bool want = false;
    while (!want && st != ST_EXIT) {
#ifdef CKMI_PHASE_TIMERS
      const int st_in = st;
      const unsigned long long t_st = __builtin_amdgcn_s_memtime();
#endif
      switch (st) {
        case ST_NEXT: {
          int r = 0;
          if (lane == 0) r = atomicAdd(queue, 1);
          r = uni(bcast(r, 0));
          if (r >= nreact) {
            st = ST_EXIT;
            break;
          }
          const int prob = io.problem[r];
          // plug flow (3) and engines (4) run in the FP64-inverse launch
          if (PF ? (sel == SEL_PFR && prob < 3) : prob >= 3) break;  // the other launch's reactor
          c.r = r;
          // TPRO runs start at the profile's initial temperature
          const double T0 = (cfg->prof_kind == 1 && cfg->energy == 2 && cfg->nprof > 0) ? cfg->prof_v[0] : io.T0[r];
          const double P0 = io.P0[r];
          double yl = 0.0;
          if (lane == 0) yl = T0;
          if (isp) yl = io.Y0[(size_t)r * KK + lane - 1];
          const double Wbar0 = 1.0 / wave_sum(isp ? yl * V.rwt()[lane - 1] : 0.0);
          if (dcfg->npe) {  // initial element contents: the element projection's target
            const uint64_t cnt = isp ? elem_table(V)[lane - 1] : 0ull;
            const double rw = isp ? V.rwt()[lane - 1] : 0.0;
            double v[PROJ_MMAX];
#pragma unroll
            for (int e = 0; e < PROJ_MMAX; ++e) v[e] = elem_coef(cnt, rw, e) * yl;
            wave_sum_multi<PROJ_MMAX>(v, lane);
#pragma unroll
            for (int e = 0; e < PROJ_MMAX; ++e) c.eb0[e] = v[e];
          }
          R.pfr = PF ? (prob == 3 ? 1 : (prob == 4 ? 2 : 0)) : 0;
          R.conp = (prob == 1 || prob == 3);
          R.energy = cfg->energy;
          R.npv = cfg->prof_kind == 0 ? cfg->nprof : 0;
          R.ntp = (cfg->prof_kind == 1 && cfg->energy == 2) ? cfg->nprof : 0;
          R.rho0 = P0 * Wbar0 / (RU * T0);
          R.V0 = (!R.conp && R.npv > 0) ? cfg->prof_v[0] : io.V0[r];
          R.P0 = (R.conp && R.npv > 0) ? cfg->prof_v[0] : P0;
          if constexpr (PF) {
            if (R.pfr == 2) {  // engine: V0 from the crank position at t = 0; gamma (G), T (Pm) of the charge
              double dv;
              engine_volume(cfg->eng, 0.0, R.V0, dv);
              const double cpR = isp ? nasa7_img(V, lane - 1, T0, log(T0), 1.0 / T0).cpR : 0.0;
              const double cpm = wave_sum(isp ? yl * cpR * V.rwt()[lane - 1] : 0.0);
              R.G = cpm / (cpm - 1.0 / Wbar0);
              R.Pm = T0;
            }
          }
          R.mass = R.rho0 * R.V0;
          if (PF && R.pfr == 1) {  // plug flow: V0 is the inlet velocity u0 [cm/s]
            R.G = R.rho0 * R.V0;  // mdot / A: the inlet density (inlet pressure) x u0, with or without PPRO
            R.Pm = R.P0 + R.G * R.V0;
          }
          R.gfac = cfg->gfac;
          R.qloss = cfg->qloss;
          R.htc = cfg->htc;
          R.areaq = cfg->areaq;
          R.tamb = cfg->tamb;
          R.nq = cfg->prof2_kind == 1 ? cfg->nprof2 : 0;
          R.na = cfg->prof2_kind == 2 ? cfg->nprof2 : cfg->nprof3;
          R.a_t = cfg->prof2_kind == 2 ? cfg->prof2_t : cfg->prof3_t;
          R.a_v = cfg->prof2_kind == 2 ? cfg->prof2_v : cfg->prof3_v;
          {
            const int ar = io.afac_rxn ? io.afac_rxn[r] : -1;
            R.pslot = (ar >= 0 && ar < img.II) ? img.slot_of[ar] : -1;
            R.plnf = R.pslot >= 0 ? log(io.afac[r]) : 0.0;
          }
          c.nadap = 0;
          c.avar_last = bcast(yl, cfg->avar > 0 ? cfg->avar : 0);
          c.T0 = T0;
          c.yguard = dcfg->guard_y;
          c.tguard_lo = dcfg->guard_tlo;
          c.tguard_hi = dcfg->guard_thi;
          S.rtol = cfg->rtol;
          S.atol = cfg->atol;
          S.nneg = cfg->nneg;
          S.ncf_tot = S.nef_tot = S.nlu = S.nfe = S.nje = S.nni = 0;
          c.tend = cfg->t_end;
          c.hmax = cfg->hmax > 0.0 ? cfg->hmax : c.tend / 100.0;
          S.hmax_inv = 1.0 / c.hmax;
          S.hmin = 0.0;
          c.ncrit = n_crit(dcfg);
          c.icrit = 0;
          c.first = 1;
          c.max_steps = cfg->max_steps > 0 ? cfg->max_steps : 200000;
#ifdef CKMI_PHASE_TIMERS
#pragma unroll
          for (int k = 0; k < 8; ++k) ph[k] = 0;
          if (lane < 40) phs[lane] = 0;
          t_r0 = __builtin_amdgcn_s_memtime();
#endif
          START_BEGIN(0.0, yl, crit_time(dcfg, c.tend, 0), cfg->h0);
          break;
        }
        case ST_START_F: {
          b.zn[1] = act ? fe : 0.0;
          S.nfe++;
          if (c.st_h0 > 0.0) {
            c.st_h = c.st_h0;
            st = ST_START_FINISH;
            break;
          }
          // initial step estimate (oracle bdf_initial_step)
          const double t0 = S.tn, tout = c.st_tout;
          const double tdist = fabs(tout - t0);
          const double tround = UROUND * fmax(fabs(t0), fabs(tout));
          const double hlb = 100.0 * tround;
          double hub = 0.1 * tdist;
          const double num = act ? fabs(b.zn[1]) : 0.0;
          const double den = 0.1 * fabs(b.zn[0]) + S.atol;
          const double hub_inv = wave_max(act ? num / (den > 0 ? den : 1e-300) : 0.0);
          if (hub * hub_inv > 1.0) hub = 1.0 / hub_inv;
          const double hg = sqrt(hlb * hub);
          if (hub < hlb) {
            c.st_h = hg;
            st = ST_START_FINISH;
            break;
          }
          c.is_t0 = t0;
          c.is_hg = hg;
          c.is_hub = hub;
          c.is_hlb = hlb;
          c.is_count = 1;
          REQUEST_F(t0 + hg, b.zn[0] + hg * b.zn[1], ST_INITSTEP_F);
          break;
        }
        case ST_INITSTEP_F: {
          S.nfe++;
          const double hg = c.is_hg, hub = c.is_hub;
          const double f1 = act ? (fe - b.zn[1]) / hg : 0.0;
          const double yddnrm = wrms_lane(f1, b.ewt, n);
          double hnew = (yddnrm * hub * hub > 2.0) ? sqrt(2.0 / yddnrm) : sqrt(hg * hub);
          bool done = c.is_count == 4;
          if (!done) {
            const double hrat = hnew / hg;
            if (hrat > 0.5 && hrat < 2.0) {
              done = true;
            } else if (c.is_count >= 2 && hrat > 2.0) {
              hnew = hg;
              done = true;
            }
          }
          if (!done) {
            c.is_hg = hnew;
            c.is_count++;
            REQUEST_F(c.is_t0 + hnew, b.zn[0] + hnew * b.zn[1], ST_INITSTEP_F);
            break;
          }
          double h0 = 0.5 * hnew;
          if (h0 < c.is_hlb) h0 = c.is_hlb;
          if (h0 > hub) h0 = hub;
          c.st_h = h0;
          st = ST_START_FINISH;
          break;
        }
        case ST_START_FINISH: {
          double h = c.st_h;
          if (h > c.hmax) h = c.hmax;
          if (h > c.st_tout - S.tn) h = c.st_tout - S.tn;
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
          st = ST_STEP_BEGIN;
          if (c.first) {
            c.first = 0;
            g.mode = cfg->ign_mode;
            g.comp = (g.mode == 4) ? 1 + cfg->ign_species : 0;
            g.found = g.started = g.have_prev = g.have_next = 0;
            g.thresh = 0.0;
            g.best = -1e300;
            g.tbest = g.tprev = g.vprev = g.tnext = g.vnext = g.tlast = g.vlast = 0.0;
            g.tau = -1.0;
            if (g.mode == 2) g.thresh = c.T0 + cfg->ign_val;
            if (g.mode == 3) g.thresh = cfg->ign_val;
            c.isave = 0;
            while (c.isave < io.nsave && io.t_save[c.isave] <= 0.0) {
              if (act) io.y_save[((size_t)c.r * io.nsave + c.isave) * n + lane] = b.zn[0];
              c.isave++;
            }
            c.status = 0;
            c.nst = 0;
            c.stopped = 0;
            if (g.mode == 1 || g.mode == 4) REQUEST_F(0.0, b.zn[0], ST_IGN0_F);
          }
          break;
        }
        case ST_IGN0_F: {
          S.nfe++;
          ign_peak_update(g, 0.0, g.mode == 1 ? bcast(fe, 0) : bcast(b.zn[0], g.comp));
          st = ST_STEP_BEGIN;
          break;
        }
        case ST_STEP_BEGIN: {
          if (!(S.tn < c.tend * (1.0 - 1e-15))) {
            st = ST_FINISH;
            break;
          }

          c.tc = crit_time(dcfg, c.tend, c.icrit);
          if (S.tn + S.hprime > c.tc) {
            const double hp = c.tc - S.tn;
            S.eta = hp / S.h;
            if (S.nst > 0) {
              S.hprime = hp;
            } else {
              bdf_rescale(b, S);
              S.hprime = S.h;
            }
          }
          b.ewt = act ? 1.0 / (S.rtol * fabs(b.zn[0]) + S.atol) : 0.0;
          c.told = S.tn;
          c.saved_t = S.tn;
          c.ncf = c.nef = 0;
          c.nflag = NF_FIRST;
          if (S.nst > 0 && S.hprime != S.h) {
            if (S.qprime != S.q) {
              bdf_adjust_order(b, S, S.qprime - S.q);
              S.q = S.qprime;
              S.L = S.q + 1;
              S.qwait = S.L;
            }
            bdf_rescale(b, S);
          }
          st = ST_STEP_ATTEMPT;
          break;
        }
        case ST_STEP_ATTEMPT: {
          bdf_predict(b, S);
          bdf_set(b, S);
          c.convfail = (c.nflag == NF_FIRST || c.nflag == NF_ERR_FAIL) ? CF_NONE : CF_OTHER;
          c.call_setup = (c.nflag != NF_FIRST) || S.nst == 0 || S.nst >= S.nstlp + MSBP || fabs(S.gamrat - 1.0) > DGMAX;
          st = ST_NLS_ATTEMPT;
          break;
        }
        case ST_NLS_ATTEMPT: {
          b.y = b.zn[0];
          REQUEST_F(S.tn, b.y, ST_NLS_F);
          break;
        }
        case ST_NLS_F: {
          b.ftemp = fe;
          S.nfe++;
          if (!c.call_setup) {
            b.acor = 0.0;
            c.delp = 0.0;
            c.mm = 0;
            st = ST_NEWTON_ITER;
            break;
          }
          const double dgamma = fabs(S.gamma / S.gammap - 1.0);
          const int jbad = S.nst == 0 || S.nst >= S.nstlj + MSBJ || (c.convfail == CF_BAD_J && dgamma < DGMAX) ||
                           c.convfail == CF_OTHER;
          if (jbad) {
            // exclusive use of the workgroup's J scratch until it is copied out
            for (;;) {
              int got = 0;
              if (lane == 0) got = atomicCAS(lds_at<int>(olock), 0, 1) == 0;
              if (uni(bcast(got, 0))) break;
              __builtin_amdgcn_s_sleep(4);
            }
            wave_lds_sync();
            REQUEST_F(S.tn, b.y, ST_NLS_J);
            with_j = true;
          } else {
            S.jcur = 0;
            st = ST_SETUP;
          }
          break;
        }
        case ST_NLS_J: {
          {
            const double* Jsh = lds_at<const double>(oJ);
#pragma unroll 2
            for (int j = 0; j < N; ++j) Jg[j * WAVE + lane] = (float)Jsh[j * LDJ + lane];
          }
          wave_lds_sync();
          if (lane == 0) atomicExch(lds_at<int>(olock), 0);
          S.nfe++;
          S.nje++;
          S.nstlj = S.nst;
          S.jcur = 1;
          st = ST_SETUP;
          break;
        }
        case ST_SETUP: {
#ifdef CKMI_PHASE_TIMERS
          const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
          // each lane reads back only the J entries it wrote itself (same-address order); the
          // dwdT row of the slice (free here) is the pivot-row scratch
          const bool ok = M.build_factor(Jg, WAVE, S.gamma, lane, n, L.base + 32 * VL);
#ifdef CKMI_PHASE_TIMERS
          ph[PH_LU] += __builtin_amdgcn_s_memtime() - t0;
#endif
          S.nlu++;
          S.crate = 1.0;
          S.gammap = S.gamma;
          S.gamrat = 1.0;
          S.nstlp = S.nst;
          if (!ok) {
            st = ST_STEP_CONVFAIL;
            break;
          }
          b.acor = 0.0;
          c.delp = 0.0;
          c.mm = 0;
          st = ST_NEWTON_ITER;
          break;
        }
        case ST_NEWTON_ITER: {
          const double rhs = act ? S.gamma * b.ftemp - (S.rl1 * b.zn[1] + b.acor) : 0.0;
#ifdef CKMI_PHASE_TIMERS
          const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
          double x = M.solve(rhs, lane, n);
#ifdef CKMI_PHASE_TIMERS
          ph[PH_SOLVE] += __builtin_amdgcn_s_memtime() - t0;
#endif
          S.nni++;
          if (S.gamrat != 1.0) x *= 2.0 / (1.0 + S.gamrat);
          if (!act) x = 0.0;
          // the iteration's norms in one fused reduction (oracle nls: the same quantities): the correction
          // (del), the accumulated correction (acnrm), NNEG's negative part and acnrm after NNEG's clipping
          const double z0 = b.zn[0];
          b.acor += x;
          b.y = z0 + b.acor;
          const bool neg = S.nneg && act && lane >= 1 && b.y < 0.0;
          double nv[4];
          {
            const double xe = x * b.ewt, ae = b.acor * b.ewt, ne = neg ? b.y * b.ewt : 0.0;
            const double fe2 = neg ? z0 * b.ewt : ae;
            nv[0] = xe * xe;
            nv[1] = ae * ae;
            nv[2] = ne * ne;
            nv[3] = fe2 * fe2;
          }
          wave_sum_multi<4>(nv, lane);
          const double del = sqrt(nv[0] / n);
          if (c.mm > 0) S.crate = fmax(CRDOWN * S.crate, del / c.delp);
          const double dcon = del * fmin(1.0, S.crate) / S.tq[4];
          if (dcon <= 1.0) {
            bool negfail = false, negfix = false;
            if (S.nneg && nv[2] > 0.0) {
              if (sqrt(nv[2] / n) > NNEG_TOL) {
                negfail = true;
              } else {
                negfix = true;
                if (neg) {
                  b.y = 0.0;
                  b.acor = -z0;
                }
              }
            }
            if (negfail) {
              c.failed = 2;
              st = ST_NLS_FAIL;
              break;
            }
            S.acnrm = (c.mm == 0 && !negfix) ? del : sqrt((negfix ? nv[3] : nv[1]) / n);
            S.jcur = 0;
            st = ST_ERRTEST;
            break;
          }
          c.mm++;
          if (c.mm == MAXCOR || (c.mm >= 2 && del > RDIV * c.delp)) {
            c.failed = 1;
            st = ST_NLS_FAIL;
            break;
          }
          c.delp = del;
          REQUEST_F(S.tn, b.y, ST_NEWTON_F);
          break;
        }
        case ST_NEWTON_F: {
          b.ftemp = fe;
          S.nfe++;
          st = ST_NEWTON_ITER;
          break;
        }
        case ST_NLS_FAIL: {
          if (c.failed == 1 && !S.jcur) {
            c.convfail = CF_BAD_J;
            c.call_setup = 1;
            st = ST_NLS_ATTEMPT;
          } else {
            st = ST_STEP_CONVFAIL;
          }
          break;
        }
        case ST_STEP_CONVFAIL: {
          c.ncf++;
          S.ncf_tot++;
          S.etamax = 1.0;
          bdf_restore(b, S, c.saved_t);
          if (fabs(S.h) <= S.hmin * ONEPSM || c.ncf == MXNCF) {
            c.rc = CKMI_RUN_CONVFAIL;
            st = ST_STEP_END;
            break;
          }
          S.eta = fmax(ETACF, S.hmin / fabs(S.h));
          c.nflag = NF_CONV_FAIL;
          bdf_rescale(b, S);
          st = ST_STEP_ATTEMPT;
          break;
        }
        case ST_ERRTEST: {
          c.dsm = S.acnrm * S.tq[2];
          if (c.dsm <= 1.0) {
            st = ST_STEP_COMPLETE;
            break;
          }
          c.nef++;
          S.nef_tot++;
          c.nflag = NF_ERR_FAIL;
          bdf_restore(b, S, c.saved_t);
          if (fabs(S.h) <= S.hmin * ONEPSM || c.nef == MXNEF) {
            c.rc = CKMI_RUN_ERRTEST;
            st = ST_STEP_END;
            break;
          }
          S.etamax = 1.0;
          st = ST_STEP_ATTEMPT;
          if (c.nef <= MXNEF1) {
            S.eta = 1.0 / (eta_root(BIAS2 * c.dsm, S.L) + ADDON);
            S.eta = fmax(ETAMIN, fmax(S.eta, S.hmin / fabs(S.h)));
            if (c.nef >= SMALL_NEF) S.eta = fmin(S.eta, ETAMXF);
            bdf_rescale(b, S);
            break;
          }
          if (S.q > 1) {
            S.eta = fmax(ETAMIN, S.hmin / fabs(S.h));
            bdf_adjust_order(b, S, -1);
            S.L = S.q;
            S.q--;
            S.qwait = S.L;
            bdf_rescale(b, S);
            break;
          }
          S.eta = fmax(ETAMIN, S.hmin / fabs(S.h));
          S.h *= S.eta;
          S.hscale = S.h;
          S.qwait = LONG_WAIT;
          REQUEST_F(S.tn, b.zn[0], ST_ERR_F);
          break;
        }
        case ST_ERR_F: {
          S.nfe++;
          b.zn[1] = act ? S.h * fe : 0.0;
          st = ST_STEP_ATTEMPT;
          break;
        }
        case ST_STEP_COMPLETE: {
          const double dsm = c.dsm;
          S.nst++;
          c.nst++;
          S.hu = S.h;
#pragma unroll
          for (int i = QMAX; i >= 2; --i)
            if (i <= S.q) S.tau[i] = S.tau[i - 1];
          if (S.q == 1 && S.nst > 1) S.tau[2] = S.tau[1];
          S.tau[1] = S.h;
          // the q - 1 and q + 1 error norms of a step that selects the next order (qwait reaches 0 below), from
          // the corrector before the element projection (oracle bdf_step), in one fused 2-value reduction
          double ddn = 0.0, dup = 0.0;
          if (S.etamax != 1.0 && S.qwait == 1) {
            const bool qm = S.q > 1, qp = S.q != QMAX && S.saved_tq5 != 0.0;
            double cquot = 0.0;
            if (qp) {
              const double hr = S.h / S.tau[2];
              double hrL = hr;
              for (int j = 1; j < S.L; ++j) hrL *= hr;
              cquot = (S.tq[5] / S.saved_tq5) * hrL;
            }
            double ov[2];
            {
              double znq = 0.0, lq = 0.0;
#pragma unroll
              for (int j = 0; j <= QMAX; ++j)
                if (j == S.q) {
                  znq = b.zn[j];
                  lq = S.l[j];
                }
              const double a = (act && qm) ? (znq + lq * b.acor) * b.ewt : 0.0;
              const double t = (act && qp) ? (b.acor - cquot * b.zn[QMAX]) * b.ewt : 0.0;
              ov[0] = a * a;
              ov[1] = t * t;
            }
            wave_sum_multi<2>(ov, lane);
            ddn = sqrt(ov[0] / n) * S.tq[1];
            dup = sqrt(ov[1] / n) * S.tq[3];
          }
          // element conservation held to PROJ_TOL rtol (oracle elem_project), before the history update
          if (dcfg->npe) elem_project_wave(V, dcfg->npe, c.eb0, S.rtol, b.zn[0], b.acor, lane, L.ek());
#pragma unroll
          for (int j = 0; j <= QMAX; ++j)
            if (j <= S.q) b.zn[j] += S.l[j] * b.acor;
          S.qwait--;
          if (S.qwait == 1 && S.q != QMAX) {
            b.zn[QMAX] = b.acor;
            S.saved_tq5 = S.tq[5];
          }
          if (S.etamax == 1.0) {
            if (S.qwait < 2) S.qwait = 2;
            S.qprime = S.q;
            S.hprime = S.h;
            S.eta = 1.0;
          } else {
            const double etaq = 1.0 / (eta_root(BIAS2 * dsm, S.L) + ADDON);
            if (S.qwait != 0) {
              S.eta = etaq;
              S.qprime = S.q;
            } else {
              S.qwait = 2;
              double etaqm1 = 0.0, etaqp1 = 0.0;
              if (S.q > 1) etaqm1 = 1.0 / (eta_root(BIAS1 * ddn, S.q) + ADDON);
              if (S.q != QMAX && S.saved_tq5 != 0.0) etaqp1 = 1.0 / (eta_root(BIAS3 * dup, S.L + 1) + ADDON);
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
          {  // runaway guard on the accepted state: a mass fraction far below 0, or T off the thermo range
             // (energy runs); it ends the reactor through ST_STEP_END's failure exit
            // (one ballot, not a max reduction: only "any lane beyond the guard" matters)
            const double z0 = b.zn[0];
            const bool bad = isp ? -z0 > c.yguard
                                 : (lane == 0 && R.energy == 1 && !(z0 >= c.tguard_lo && z0 <= c.tguard_hi));
            c.rc = __ballot(bad) != 0 ? CKMI_RUN_RUNAWAY : 0;
          }
          if constexpr (PF) {  // plug flow past the choke point of the momentum equation (pfr_pressure)
            if (R.pfr == 1 && R.npv == 0 && c.rc == 0) {
              const double z0 = b.zn[0];
              const double sYW = wave_sum(isp ? z0 * V.rwt()[lane - 1] : 0.0);
              if (R.Pm * R.Pm - 4.0 * R.G * R.G * RU * bcast(z0, 0) * sYW < 0.0) c.rc = CKMI_RUN_CHOKED;
            }
          }
          st = ST_STEP_END;
          break;
        }
        case ST_STEP_END: {
          if (c.rc != 0) {
            c.status = c.rc;
            st = ST_FINISH;
            break;
          }
          const double tn = S.tn;
          while (c.isave < io.nsave && io.t_save[c.isave] <= tn) {
            const double ys = dky0_lane(b, S, io.t_save[c.isave]);
            if (act) io.y_save[((size_t)c.r * io.nsave + c.isave) * n + lane] = ys;
            c.isave++;
          }
          if (g.mode == 1) {
            ign_peak_update(g, tn, bcast(b.zn[1], 0) / S.h);
          } else if (g.mode == 4) {
            ign_peak_update(g, tn, bcast(b.zn[0], g.comp));
          } else if ((g.mode == 2 || g.mode == 3) && !g.found && bcast(b.zn[0], 0) >= g.thresh) {
            double lo = c.told, hi = tn;
            for (int it = 0; it < 60; ++it) {
              const double mid = 0.5 * (lo + hi);
              if (bcast(dky0_lane(b, S, mid), 0) >= g.thresh) hi = mid;
              else lo = mid;
            }
            g.found = 1;
            g.tau = hi;
          }
          st = ST_STEP_BEGIN;
          if (cfg->ign_stop) {
            if ((g.mode == 2 || g.mode == 3) && g.found) {
              c.stopped = 1;
              st = ST_FINISH;
              break;
            }
            if (g.mode == 1 && g.have_next && g.vlast < 0.1 * g.best && bcast(b.zn[0], 0) > c.T0 + 200.0) {
              c.stopped = 1;
              st = ST_FINISH;
              break;
            }
          }
          bool adap = false;
          if (io.n_adap && c.nadap < io.max_adap) {
            // ADAP: extra solution points every ASTEPS steps, or when AVAR moved by AVALUE
            if (cfg->asteps > 0 && c.nst % cfg->asteps == 0) adap = true;
            if (cfg->avar >= 0 && cfg->avalue > 0.0) {
              const double v = bcast(b.zn[0], cfg->avar);
              if (fabs(v - c.avar_last) >= cfg->avalue) adap = true;
            }
          }
          if (adap) {
            const size_t a = (size_t)c.r * io.max_adap + c.nadap;
            if (lane == 0) io.t_adap[a] = tn;
            if (act) io.y_adap[a * n + lane] = b.zn[0];
            c.nadap++;
            if (cfg->avar >= 0) c.avar_last = bcast(b.zn[0], cfg->avar);
          }
          if (c.nst >= c.max_steps) {
            c.status = CKMI_RUN_MAXSTEPS;
            st = ST_FINISH;
            break;
          }
          if (tn >= c.tc * (1.0 - 1e-15) && c.icrit < c.ncrit - 1) {
            c.icrit++;
            START_BEGIN(tn, b.zn[0], crit_time(dcfg, c.tend, c.icrit), 0.0);
          }
          break;
        }
        case ST_FINISH: {
          double yf;
          double tf = c.tend;
          if (c.stopped || c.status) {
            tf = S.tn;
            yf = b.zn[0];
          } else {
            yf = dky0_lane(b, S, c.tend);
          }
          if (g.mode == 1 || g.mode == 4) g.tau = ign_peak_time(g);
          double Pf, Vf;
          state_PV<PF>(V, R, tf, yf, lane, Pf, Vf);
          const int r = c.r;
          // a run that ended early (IGN_STOP, solver failure) has no solution after tf: its
          // remaining DTSV rows are NaN, never stale memory (the host trims them)
          while (c.isave < io.nsave) {
            if (act) io.y_save[((size_t)r * io.nsave + c.isave) * n + lane] = __builtin_nan("");
            c.isave++;
          }
          if (io.t_stop && lane == 0) io.t_stop[r] = tf;
          if (lane == 0) {
            io.tau[r] = g.tau;
            io.T[r] = yf;
            io.P[r] = Pf;
            io.V[r] = Vf;
            int* sto = io.stats + (size_t)r * CKMI_NSTAT;
            sto[CKMI_STAT_NST] = c.nst;
            sto[CKMI_STAT_NFE] = S.nfe;
            sto[CKMI_STAT_NJE] = S.nje;
            sto[CKMI_STAT_NLU] = S.nlu;
            sto[CKMI_STAT_NCF] = S.ncf_tot;
            sto[CKMI_STAT_NEF] = S.nef_tot;
            sto[CKMI_STAT_STATUS] = c.status;
            sto[CKMI_STAT_NNI] = S.nni;
          }
          if (isp) io.Y[(size_t)r * KK + lane - 1] = yf;
          if (io.n_adap && lane == 0) io.n_adap[r] = c.nadap;
#ifdef CKMI_PHASE_TIMERS
          ph[PH_TOTAL] = __builtin_amdgcn_s_memtime() - t_r0;
          wave_lds_sync();
          if (g_phase_buf && lane < PH_N) {
            unsigned long long v = lane >= PH_STATE ? phs[lane - PH_STATE] : 0;
#pragma unroll
            for (int k = 0; k < 8; ++k) v = (lane == k) ? ph[k] : v;
            g_phase_buf[(size_t)r * PH_N + lane] = v;
          }
#endif
          st = ST_NEXT;
          break;
        }
        default:
          st = ST_EXIT;
          break;
      }
#ifdef CKMI_PHASE_TIMERS
      if (st_in != ST_NEXT && st_in != ST_FINISH && lane == 0) phs[st_in] += __builtin_amdgcn_s_memtime() - t_st;
#endif
    }
    if (st == ST_EXIT) break;
    // the single RHS (+ Jacobian) evaluation site of the integrator
#ifdef CKMI_PHASE_TIMERS
    const unsigned long long t0 = __builtin_amdgcn_s_memtime();
#endif
#ifdef CKMI_PHASE_TIMERS
    unsigned long long sub[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    fe = reactor_rhs<PL, PF>(V, R, t_e, y_e, L, oJ, lane, N, with_j, sub);
    ph[with_j ? PH_JAC : PH_RHS] += __builtin_amdgcn_s_memtime() - t0;
    if (!with_j) {
      ph[5] += sub[0];
      ph[6] += sub[1];
      ph[7] += sub[2];
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 6; ++k) phs[24 + k] += sub[3 + k];
      }
    }
#else
    fe = reactor_rhs<PL, PF>(V, R, t_e, y_e, L, oJ, lane, N, with_j);
#endif
  }
#undef REQUEST_F
#undef START_BEGIN
}

// ---------------------------------------------------------------- engine heat release
// Heat rates of an engine run on its saved states (KINAll0D_GetEngineHeatRelease, engine.py:953-988):
// one wave per state evaluates the integrator's own right-hand side (reactor_rhs, problem 4) there,
// so the rates are the ones the solution was integrated with, not finite differences of it:
//   ahrr  = m c_v dT/dt + P dV/dt   [erg/s]  apparent heat release (chemical heat release net of the
//                                           wall loss: the first law of the closed cylinder)
//   qloss = hA (T - T_wall)          [erg/s]  wall heat loss (ICHX / Woschni, engine_hA; 0 adiabatic)
// The per-reactor context is built from the cylinder's initial state as the reactor kernel does.
template <bool PL>
__global__ __launch_bounds__(WAVE) void engine_heat_kernel(MechImage img, const DevCfg* __restrict__ dcfg, double T0,
                                                           double P0, const double* __restrict__ Y0, int n,
                                                           const double* __restrict__ ts, const double* __restrict__ ys,
                                                           double* __restrict__ ahrr, double* __restrict__ qloss) {
  const ckmi_reactor_cfg* __restrict__ cfg = &dcfg->c;
  stage_image(0, img);
  const MechView V = make_view(0, img);
  const int lane = threadIdx.x;
  WaveLds L;
  L.base = align16(img.bytes);
  RunCtx& R = *lds_at<RunCtx>(L.base + slice_vec_bytes(img.G));
  const int KK = V.KK;
  const bool isp = lane >= 1 && lane <= KK;
  const int s = isp ? lane - 1 : 0;
  const double rw = isp ? V.rwt()[s] : 0.0;
  const double y0 = lane == 0 ? T0 : (isp ? Y0[s] : 0.0);
  const double Wbar0 = 1.0 / wave_sum(isp ? y0 * rw : 0.0);
  if (lane == 0) {
    R.cfg = cfg;
    R.pfr = 2;
    R.conp = 0;
    R.energy = cfg->energy;
    R.npv = 0;
    R.ntp = 0;
    R.rho0 = P0 * Wbar0 / (RU * T0);
    double dv;
    engine_volume(cfg->eng, 0.0, R.V0, dv);
    R.P0 = P0;
    R.mass = R.rho0 * R.V0;
    R.gfac = cfg->gfac;
    R.qloss = R.htc = R.areaq = 0.0;
    R.tamb = 300.0;
    R.nq = R.na = 0;
    R.a_t = R.a_v = nullptr;
    R.pslot = -1;
    R.plnf = 0.0;
  }
  {  // gamma of the charge (Woschni's motored pressure) and its temperature, as the reactor kernel
    const double cpR = isp ? nasa7_img(V, s, T0, log(T0), 1.0 / T0).cpR : 0.0;
    const double cpm = wave_sum(isp ? y0 * cpR * rw : 0.0);
    if (lane == 0) {
      R.G = cpm / (cpm - 1.0 / Wbar0);
      R.Pm = T0;
    }
  }
  wave_lds_sync();
  for (int i = blockIdx.x; i < n; i += gridDim.x) {
    const double t = ts[i];
    const double yl = lane <= KK ? ys[(size_t)i * (KK + 1) + lane] : 0.0;
    if (lane == 0) R.tsel = t;
    wave_lds_sync();
#ifdef CKMI_PHASE_TIMERS
    unsigned long long sub[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
    const double fl = reactor_rhs<PL, true>(V, R, t, yl, L, 0, lane, WAVE, false, sub);
#else
    const double fl = reactor_rhs<PL, true>(V, R, t, yl, L, 0, lane, WAVE, false);
#endif
    const double T = bcast(yl, 0), dTdt = bcast(fl, 0);
    const double Yk = isp ? yl : 0.0;
    const double lnT = log(T);
    const Thermo7 th = isp ? nasa7_img(V, s, T, lnT, 1.0 / T) : Thermo7{0.0, 0.0, 0.0};
    const double cpk = th.cpR * RU * rw;
    const double cvm = wave_sum(Yk * (cpk - RU * rw));
    const double Wbar = 1.0 / wave_sum(Yk * rw);
    double Vc, dVdt;
    engine_volume(cfg->eng, t, Vc, dVdt);
    const double rho = R.mass / Vc;
    const double P = rho * RU * T / Wbar;
    double q = 0.0;
    if (cfg->eng[CKMI_ENG_HTMODEL] == 1.0) {  // the RHS's wall term (reactor_rhs, engine branch)
      const double cpmass = wave_sum(Yk * cpk);
      const double xp = fmax(Yk, 0.0) * rw;
      const double Tw = cfg->eng[CKMI_ENG_TWALL];
      q = engine_hA(V, R, T, log(0.5 * (T + Tw)), P, rho, Vc, xp / wave_sum(xp), cpmass, isp, s) * (T - Tw);
    }
    if (lane == 0) {
      ahrr[i] = R.mass * cvm * dTdt + P * dVdt;
      qloss[i] = q;
    }
    wave_lds_sync();  // R.tsel and the slice are rewritten for the next state
  }
}

// ---------------------------------------------------------------- ROP kernels
// Persistent grid of ROP_WAVES-wave workgroups; the workgroup stages the mechanism image in LDS
// once, each wave then takes tasks of ROP_CHUNK consecutive states and evaluates them one at a
// time (lanes over species for thermo, over reactions for the rates).  Consecutive states of one
// wave touch the same cache lines of the species-major inputs / outputs ([KK][n]), so each line
// is fetched once by one XCD and partial-line writes merge in its L2 (one state per workgroup
// spread consecutive states over all 8 XCDs: 4-8x HBM traffic, measured).
//
// Inputs and outputs of a chunk move through LDS in half-chunks of ROP_SUB states: rows T, P,
// Y_1..Y_KK of ROP_SUB consecutive states are loaded with one 64-B request per row, and the
// half-chunk's wdot_1..wdot_KK, cp, h go back the same way, so every HBM request covers whole
// 64-B halves of 128-B lines (one state at a time, lane = species, touched 53 lines with 8 B
// each: 8.8x the algorithmic traffic, measured).
//
// Mechanisms with more than 63 species (up to 255) run the same kernel with NCH = KKp / 64
// species per lane (lane + 64 j) and half as many waves per workgroup (the image, the species
// arrays and the staging rows grow with KK).
constexpr int ROP_WAVES = 8;
constexpr int ROP_CHUNK = 16;
constexpr int ROP_SUB = 8;
constexpr int ROP_LD = ROP_SUB + 1;  // odd row stride: lane = species reads of one state spread over the banks
__host__ __device__ constexpr int rop_waves(int nch) { return nch == 1 ? ROP_WAVES : 4; }
__host__ __device__ constexpr int rop_io_bytes(int KK) { return align16(8 * ROP_LD * (KK + 2)); }
__host__ __device__ constexpr int rop_slice_bytes(int G, int KK, int KKp) {
  return align16(8 * (3 * KKp + (G > 0 ? G : 1))) + rop_io_bytes(KK);
}

template <int MODE, int NCH, bool PL = false>  // MODE 0: wdot + cp + h, 1: qf / qr; NCH species per lane; PL: PLOG
__global__ __launch_bounds__(rop_waves(NCH)* WAVE) void rop_kernel(MechImage img, const int* __restrict__ orig,
                                                                  int nstate, const double* __restrict__ Tv,
                                                                  const double* __restrict__ Pv,
                                                                  const double* __restrict__ Yv,
                                                                  double* __restrict__ o0, double* __restrict__ o1,
                                                                  double* __restrict__ o2) {
  constexpr int NW = rop_waves(NCH);
  stage_image(0, img);
  const MechView V = make_view(0, img);
  const int wid = threadIdx.x / WAVE;
  const int lane = threadIdx.x % WAVE;
  const int KKp = img.KKp;
  const int slice = rop_slice_bytes(img.G, img.KK, KKp);
  const int oC = img.bytes + wid * slice;
  double* C = lds_at<double>(oC);
  double* gRT = C + KKp;
  double* wdot = gRT + KKp;
  double* Mg = wdot + KKp;
  const int KK = V.KK;
  const int sp_one = img.sp_one;
  // half-chunk staging rows [KK + 2][ROP_SUB]: T, P, Y_k in; cp, h, wdot_k out (same slots)
  double* io = lds_at<double>(oC + slice - rop_io_bytes(img.KK));
  const int nrow = KK + 2;
  const int io_c = lane & (ROP_SUB - 1), io_r = lane / ROP_SUB;
  double rw[NCH];
#pragma unroll
  for (int j = 0; j < NCH; ++j) rw[j] = lane + WAVE * j < KK ? V.rwt()[lane + WAVE * j] : 0.0;
  const int ntask = (nstate + ROP_CHUNK - 1) / ROP_CHUNK;
  for (int task = blockIdx.x * NW + wid; task < ntask; task += gridDim.x * NW) {
    const int s1 = min(nstate, (task + 1) * ROP_CHUNK);
    for (int st = task * ROP_CHUNK; st < s1; ++st) {
      const int c = st & (ROP_SUB - 1);
      const int sb = st - c;                      // first state of this half-chunk
      const int cnt = min(ROP_SUB, s1 - sb);      // states in it
      if (c == 0) {
        for (int r = io_r; r < nrow; r += WAVE / ROP_SUB) {
          double v = 0.0;
          if (io_c < cnt) v = r == 0 ? Tv[sb + io_c] : (r == 1 ? Pv[sb + io_c] : Yv[(size_t)(r - 2) * nstate + sb + io_c]);
          io[r * ROP_LD + io_c] = v;
        }
        wave_lds_sync();
      }
      const double T = io[c], P = io[ROP_LD + c];
      double yk[NCH];
      double syw = 0.0;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int k = lane + WAVE * j;
        yk[j] = k < KK ? io[(2 + k) * ROP_LD + c] : 0.0;
        syw = fma(yk[j], rw[j], syw);
      }
      const double sumYW = wave_sum(syw);
      const double rho = P / (RU * T * sumYW);
      const double lnT = log(T), invT = 1.0 / T, lnPRT = LN_PATM_RU - lnT;
      double cpm = 0.0, hm = 0.0;
#pragma unroll
      for (int j = 0; j < NCH; ++j) {
        const int k = lane + WAVE * j;
        if (k < KK) {
          const Thermo7 th = nasa7_img(V, k, T, lnT, invT);
          C[k] = rho * yk[j] * rw[j];
          gRT[k] = th.hRT - th.sR;
          wdot[k] = 0.0;
          cpm += yk[j] * th.cpR * RU * rw[j];
          hm += yk[j] * th.hRT * RU * T * rw[j];
        } else if (k == sp_one) {
          C[sp_one] = 1.0;
          gRT[sp_one] = 0.0;
        }
      }
      const double Ctot = rho * sumYW;
      wave_lds_sync();
      for (int g = lane; g < V.G; g += WAVE) {
        double m = Ctot;
        for (int p = V.gptr()[g]; p < V.gptr()[g + 1]; ++p) m += V.geff()[p] * C[V.gsp()[p]];
        Mg[g] = m;
      }
      wave_lds_sync();
      for (int base = 0; base < V.IIp; base += WAVE) {
        const int i = base + lane;
        const uint32_t inf = V.info()[i];
        const int nr = rx_nr(inf), np = rx_np(inf);
        if constexpr (PL) {
          if (inf & RX_GEN) {  // FORD / RORD / non-integral coefficients
            const double* g;
            const Rxn e = eval_gen_img(V, i, inf, T, lnT, invT, lnPRT, P, C, gRT, gRT, Mg, false, -1, 0.0, 1.0, g);
            const double qf = e.mfac * e.kf * e.pf, qr = e.mfac * e.kr * e.pr;
            if (MODE == 1) {
              const int oi = orig[i];
              o0[(size_t)oi * nstate + st] = qf;
              o1[(size_t)oi * nstate + st] = qr;
            } else {
              const double q = qf - qr;
              for (int u = 0; u < (int)g[0]; ++u) atomicAdd(&wdot[(int)g[2 + 3 * u]], -g[3 + 3 * u] * q);
              for (int u = 0; u < (int)g[1]; ++u) atomicAdd(&wdot[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * q);
            }
            continue;
          }
        }
        if (nr + np == 0) continue;
        const uint32_t rs = V.rsp()[i], ps = V.psp()[i];
        const Rxn e = eval_rxn_img<PL>(V, i, inf, rs, ps, 0u, T, lnT, invT, lnPRT, P, C, gRT, gRT, Mg, false);
        const double qf = e.mfac * e.kf * e.pf, qr = e.mfac * e.kr * e.pr;
        if (MODE == 1) {
          const int oi = orig[i];
          o0[(size_t)oi * nstate + st] = qf;
          o1[(size_t)oi * nstate + st] = qr;
        } else {
          const double q = qf - qr;
          const bool s23 = __ballot(nr > 2 || np > 2) != 0;
#pragma unroll
          for (int u = 0; u < 4; ++u) {
            if (u >= 2 && !s23) break;
            if (u < nr) atomicAdd(&wdot[sp_of(rs, u)], -q);
            if (u < np) atomicAdd(&wdot[sp_of(ps, u)], q);
          }
        }
      }
      if (MODE == 0) {
        wave_lds_sync();
#pragma unroll
        for (int j = 0; j < NCH; ++j) {
          const int k = lane + WAVE * j;
          if (k < KK) io[(2 + k) * ROP_LD + c] = wdot[k];
        }
        const double cps = wave_sum(cpm), hs = wave_sum(hm);
        if (lane == 0) {
          io[c] = cps;
          io[ROP_LD + c] = hs;
        }
      }
      wave_lds_sync();  // the next state overwrites C / gRT / wdot
      if (MODE == 0 && (c == cnt - 1)) {
        for (int r = io_r; r < nrow; r += WAVE / ROP_SUB) {
          if (io_c < cnt) {
            const double v = io[r * ROP_LD + io_c];
            if (r >= 2) o0[(size_t)(r - 2) * nstate + sb + io_c] = v;
            else if (r == 0 && o1) o1[sb + io_c] = v;
            else if (r == 1 && o2) o2[sb + io_c] = v;
          }
        }
        wave_lds_sync();  // the next half-chunk's loads overwrite io
      }
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

// ---------------------------------------------------------------- LDS lane assignment
// The reaction strips scatter each lane's rate into the wave's wdot[] with one LDS atomic per unit
// slot (reactor_rhs, rop_kernel) and gather C[] / g/RT[] through the same slots.  Which reaction sits
// on which lane of its (type, slot-class) block, and in which order a reaction's unit slots are
// listed, are free choices (products and sums over the slots commute); they decide the LDS bank
// conflicts: ds_add_f64 is serviced in 16-lane groups on banks (a/4) mod 32, so two lanes of a group
// adding to one species (or to species k and k + 16) serialise; ds_read_b64 in 32-lane groups on
// banks (a/4) mod 64, where distinct species k and k + 32 collide.  Common species (H, O, OH, H2O)
// make the mechanism's file order 4x conflict-bound (GRI-3.0: 456 LDS cycles of atomics per RHS
// against 108 conflict-free, model below).  A deterministic annealing over lane swaps within a block
// and slot orders within a reaction minimises the modelled cycles; the device code is unchanged.
namespace lanes {
struct Rx {
  int ns[2];        // unit slots per side (a species with coefficient c occupies c slots)
  uint8_t sp[2][4]; // the slots' species
};
// modelled LDS cycles of one strip (64 lanes): atomics (16-lane groups, max bank multiplicity) +
// two gathers per slot (32-lane groups, max distinct addresses per bank)
static int strip_cost(const std::vector<Rx>& rx, const std::vector<int>& lane_rx, int s0) {
  bool s23 = false;
  for (int l = 0; l < WAVE; ++l) {
    const int r = lane_rx[s0 + l];
    if (r >= 0 && (rx[r].ns[0] > 2 || rx[r].ns[1] > 2)) s23 = true;
  }
  int cost = 0;
  for (int side = 0; side < 2; ++side)
    for (int u = 0; u < (s23 ? 4 : 2); ++u) {
      for (int g0 = 0; g0 < WAVE; g0 += 16) {  // atomics
        int mult[32] = {0}, mx = 0;
        for (int l = g0; l < g0 + 16; ++l) {
          const int r = lane_rx[s0 + l];
          if (r < 0 || u >= rx[r].ns[side]) continue;
          mx = std::max(mx, ++mult[(2 * rx[r].sp[side][u]) & 31]);
        }
        cost += mx;
      }
      for (int g0 = 0; g0 < WAVE; g0 += 32) {  // gathers (C and g/RT: counted twice)
        int seen[64];
        int nseen = 0, mult[64] = {0}, mx = 0;
        for (int l = g0; l < g0 + 32; ++l) {
          const int r = lane_rx[s0 + l];
          if (r < 0 || u >= rx[r].ns[side]) continue;
          const int k = rx[r].sp[side][u];
          bool dup = false;
          for (int q = 0; q < nseen; ++q) dup |= seen[q] == k;
          if (dup) continue;
          seen[nseen++] = k;
          mx = std::max(mx, ++mult[(2 * k) & 63]);
        }
        cost += 2 * mx;
      }
    }
  return cost;
}
}  // namespace lanes

// slots: device slot -> original reaction (-1 pad), reordered in place within (rtype, slot class)
// blocks; perm[i]: the unit-slot order of original reaction i (reactant slots 0..3, product 4..7)
void assign_lanes(const ckmi_mech_desc* d, std::vector<int>& slots, const std::vector<int>& blk,
                  std::vector<std::array<uint8_t, 8>>& perm) {
  using lanes::Rx;
  const int II = d->II, n = (int)slots.size();
  std::vector<Rx> rx(II);
  perm.assign(II, {0, 1, 2, 3, 0, 1, 2, 3});
  for (int i = 0; i < II; ++i) {
    Rx& r = rx[i];
    for (int side = 0; side < 2; ++side) {
      const int ns = side == 0 ? d->nr[i] : d->np[i];
      const int32_t* sp = (side == 0 ? d->rsp : d->psp) + CKMI_SLOTS * i;
      const double* nu = (side == 0 ? d->rnu : d->pnu) + CKMI_SLOTS * i;
      int c = 0;
      for (int u = 0; u < ns && !rxn_general(d, i); ++u)
        for (int k = 0; k < (int)nu[u] && c < 4; ++k) r.sp[side][c++] = (uint8_t)sp[u];
      r.ns[side] = rxn_general(d, i) ? 0 : c;
    }
  }
  const int nstrip = n / WAVE;
  std::vector<int> cost(nstrip);
  for (int s = 0; s < nstrip; ++s) cost[s] = lanes::strip_cost(rx, slots, s * WAVE);
  uint64_t st = 0x9e3779b97f4a7c15ull;  // deterministic: the same image on every run and device
  auto rnd = [&]() {
    st ^= st << 13, st ^= st >> 7, st ^= st << 17;
    return st;
  };
  double temp = 2.0;
  // 400 proposals per slot, capped at 1024 slots' worth: mechanisms of thousands of reactions would
  // otherwise spend seconds of host time per ckmi_mech_create (round-4 advice); the GRI-3.0 (384 slots)
  // and 161-species (512) images are annealed exactly as before
  const int iters = 400 * std::min(n, 1024);
  for (int it = 0; it < iters; ++it, temp = std::max(0.05, temp * (1.0 - 6.0 / iters))) {
    const int a = (int)(rnd() % n);
    if (slots[a] < 0) continue;
    int b = -1;
    Rx save_a = rx[slots[a]];
    if (rnd() & 1) {  // swap two lanes of one block
      b = (int)(rnd() % n);
      if (b == a || slots[b] < 0 || blk[slots[b]] != blk[slots[a]]) continue;
      std::swap(slots[a], slots[b]);
    } else {  // swap two unit slots of one side of one reaction
      Rx& r = rx[slots[a]];
      const int side = (int)(rnd() & 1);
      if (r.ns[side] < 2) continue;
      const int u = (int)(rnd() % r.ns[side]), v = (int)(rnd() % r.ns[side]);
      if (u == v || r.sp[side][u] == r.sp[side][v]) continue;
      std::swap(r.sp[side][u], r.sp[side][v]);
    }
    const int sa = a / WAVE, sb = b >= 0 ? b / WAVE : sa;
    const int ca = lanes::strip_cost(rx, slots, sa * WAVE), cb = sb != sa ? lanes::strip_cost(rx, slots, sb * WAVE) : 0;
    const int delta = ca + cb - cost[sa] - (sb != sa ? cost[sb] : 0);
    const double x = (double)(rnd() >> 11) * (1.0 / 9007199254740992.0);
    if (delta <= 0 || x < std::exp(-delta / temp)) {
      cost[sa] = ca;
      if (sb != sa) cost[sb] = cb;
    } else if (b >= 0) {
      std::swap(slots[a], slots[b]);
    } else {
      rx[slots[a]] = save_a;
    }
  }
  // the slot orders as permutations of the file's unit-slot expansion
  for (int i = 0; i < II; ++i) {
    Rx ref;
    for (int side = 0; side < 2; ++side) {
      const int ns = side == 0 ? d->nr[i] : d->np[i];
      const int32_t* sp = (side == 0 ? d->rsp : d->psp) + CKMI_SLOTS * i;
      const double* nu = (side == 0 ? d->rnu : d->pnu) + CKMI_SLOTS * i;
      int c = 0;
      for (int u = 0; u < ns && !rxn_general(d, i); ++u)
        for (int k = 0; k < (int)nu[u] && c < 4; ++k) ref.sp[side][c++] = (uint8_t)sp[u];
      bool used[4] = {false, false, false, false};
      for (int u = 0; u < rx[i].ns[side]; ++u)
        for (int v = 0; v < rx[i].ns[side]; ++v)
          if (!used[v] && ref.sp[side][v] == rx[i].sp[side][u]) {
            used[v] = true;
            perm[i][4 * side + u] = (uint8_t)v;
            break;
          }
    }
  }
}

// Pack the compact mechanism image (ckmi_image.hpp) from the device-slot tables.
int build_image(ckmi_mech* m, const ckmi_mech_desc* d, const std::vector<int>& slots, const std::vector<int>& flags,
                const std::vector<int>& nrp, const std::vector<int4>& rsp, const std::vector<int4>& psp,
                const std::vector<double>& rnu, const std::vector<double>& pnu, const std::vector<double>& lnA,
                const std::vector<double>& beta, const std::vector<double>& Ea, const std::vector<double>& lnA0,
                const std::vector<double>& beta0, const std::vector<double>& Ea0, const std::vector<double>& fp,
                const std::vector<double>& rlnA, const std::vector<double>& rbeta, const std::vector<double>& rEa,
                const std::vector<int>& tb, const std::vector<int>& gptr, const std::vector<int>& gsp,
                const std::vector<double>& geff, const std::vector<double>& wt, const std::vector<double>& rwt,
                const std::vector<std::array<uint8_t, 8>>& perm) {
  const int KK = m->KK, IIp = m->IIpad, G = m->G;
  const int KKp = (KK + 1 + WAVE - 1) / WAVE * WAVE;  // room for the dummy species slot
  const int sp_one = KKp - 1;                          // = SP_ONE (63) whenever KK <= 63
  if (KK > KK_IMAGE_MAX)
    return fail(CKMI_ERR_UNSUPPORTED, "more than 255 species not supported by the mechanism image");
  std::vector<uint32_t> urs(IIp, 0), ups(IIp, 0), unu(IIp, 0), uinfo(IIp, 0);
  std::vector<double> aux;
  int naux = 0;
  for (int s = 0; s < IIp; ++s) {
    const int nr = nrp[s] & 0xff, np = nrp[s] >> 8;
    uint32_t a = 0, b = 0, nu = 0;
    const int* r4 = &rsp[s].x;
    const int* p4 = &psp[s].x;
    const bool gen = (flags[s] & RX_GEN) != 0;  // real coefficients: no unit slots, aux stream
    // unit-coefficient slots: a species with coefficient c occupies c slots
    int ns_r = 0, ns_p = 0;
    int ur[4] = {0, 0, 0, 0}, up[4] = {0, 0, 0, 0};  // unit slots in file order, then in assign_lanes' order
    for (int u = 0; u < nr && !gen; ++u) {
      const int c = (int)rnu[u * IIp + s];
      nu |= (uint32_t)std::min(c, 15) << (4 * u);
      for (int k = 0; k < c; ++k, ++ns_r)
        if (ns_r < 4) ur[ns_r] = r4[u];
    }
    for (int u = 0; u < np && !gen; ++u) {
      const int c = (int)pnu[u * IIp + s];
      nu |= (uint32_t)std::min(c, 15) << (16 + 4 * u);
      for (int k = 0; k < c; ++k, ++ns_p)
        if (ns_p < 4) up[ns_p] = p4[u];
    }
    if (ns_r > 4 || ns_p > 4)
      return fail(CKMI_ERR_UNSUPPORTED, "more than 4 molecules (sum of coefficients) on a reaction side");
    const uint8_t* pm = slots[s] >= 0 ? perm[slots[s]].data() : nullptr;
    for (int u = 0; u < ns_r; ++u) a |= (uint32_t)ur[pm ? pm[u] : u] << (8 * u);
    for (int u = 0; u < ns_p; ++u) b |= (uint32_t)up[pm ? pm[4 + u] : u] << (8 * u);
    for (int u = ns_r; u < 4; ++u) a |= (uint32_t)sp_one << (8 * u);
    for (int u = ns_p; u < 4; ++u) b |= (uint32_t)sp_one << (8 * u);
    urs[s] = a;
    ups[s] = b;
    unu[s] = nu;
    const int fl = flags[s];
    const int type = fl & 3;
    uint32_t inf = (uint32_t)(fl & 0x7f) | ((uint32_t)ns_r << 7) | ((uint32_t)ns_p << 10) | (uint32_t)(fl & 0x2000) |
                   (uint32_t)(fl & RX_GEN) | (uint32_t)(fl & RX_ALT);
    if (slots[s] >= 0 && type == CKMI_RXN_PLOG && (fl & RX_ALT)) {
      // Chebyshev stream: NT, NP, 1/Tmin, 1/Tmax, log10 Pmin, log10 Pmax [dyn/cm2], then a[t][p]
      const int i = slots[s];
      const double* r = d->plog_par + 4 * d->plog_ptr[i];
      const int nt = (int)r[0], npr = (int)r[1];
      std::vector<double> rec{(double)nt, (double)npr, 1.0 / r[4], 1.0 / r[5], std::log10(r[6] * 1.01325e6),
                              std::log10(r[7] * 1.01325e6)};
      rec.insert(rec.end(), r + 8, r + 8 + nt * npr);
      rec.resize((rec.size() + AUXW - 1) / AUXW * AUXW, 0.0);
      aux.insert(aux.end(), rec.begin(), rec.end());
      inf |= (uint32_t)naux << 16;
      naux += (int)rec.size() / AUXW;
    } else if (slots[s] >= 0 && type == CKMI_RXN_PLOG) {
      // PLOG stream: npts, then (ln P, ln A, b, E/R) per point, over ceil((1 + 4 npts) / AUXW) records
      const int i = slots[s], p0 = d->plog_ptr[i], n = d->plog_ptr[i + 1] - p0;
      std::vector<double> rec{(double)n};
      rec.insert(rec.end(), d->plog_par + 4 * p0, d->plog_par + 4 * (p0 + n));
      rec.resize((rec.size() + AUXW - 1) / AUXW * AUXW, 0.0);
      aux.insert(aux.end(), rec.begin(), rec.end());
      inf |= (uint32_t)naux << 16;
      naux += (int)rec.size() / AUXW;
    } else if (slots[s] >= 0 && (type == 2 || (fl & 8) || gen || (fl & RX_ALT))) {
      // (a Landau-Teller reaction's record: low = B, C of LT; fp[0], fp[1] = B, C of RLT)
      double rec[AUXW] = {lnA0[s], beta0[s], Ea0[s], fp[0 * IIp + s], fp[1 * IIp + s], fp[2 * IIp + s],
                          fp[3 * IIp + s], fp[4 * IIp + s], rlnA[s], rbeta[s], rEa[s], 0.0};
      const int ft = (fl >> 4) & 7;
      if (ft == CKMI_FALL_TROE3 || ft == CKMI_FALL_TROE4) {  // exp(-T / T***), exp(-T / T*): store 1/T
        rec[4] = 1.0 / rec[4];
        rec[5] = 1.0 / rec[5];
      } else if (ft == CKMI_FALL_SRI) {  // exp(-T / c)
        rec[5] = 1.0 / rec[5];
      }
      aux.insert(aux.end(), rec, rec + AUXW);
      inf |= (uint32_t)naux << 16;
      ++naux;
      if (gen) {  // records naux..: nr, np, (species, nu, order) x 4 reactant and x 4 product slots
        const int i = slots[s];
        double grec[GEN_RECORDS * AUXW] = {(double)nr, (double)np};
        for (int u = 0; u < nr; ++u) {
          grec[2 + 3 * u] = d->rsp[CKMI_SLOTS * i + u];
          grec[3 + 3 * u] = d->rnu[CKMI_SLOTS * i + u];
          grec[4 + 3 * u] = d->ford ? d->ford[CKMI_SLOTS * i + u] : d->rnu[CKMI_SLOTS * i + u];
        }
        for (int u = 0; u < np; ++u) {
          grec[GEN_P + 3 * u] = d->psp[CKMI_SLOTS * i + u];
          grec[GEN_P + 1 + 3 * u] = d->pnu[CKMI_SLOTS * i + u];
          grec[GEN_P + 2 + 3 * u] = d->rord ? d->rord[CKMI_SLOTS * i + u] : d->pnu[CKMI_SLOTS * i + u];
        }
        aux.insert(aux.end(), grec, grec + GEN_RECORDS * AUXW);
        naux += GEN_RECORDS;
      }
    }
    uinfo[s] = inf;
  }
  if (naux == 0) aux.assign(AUXW, 0.0), naux = 1;
  std::vector<double> th(15 * KKp, 0.0), wtp(KKp, 0.0), rwtp(KKp, 0.0);
  for (int k = 0; k < KK; ++k) {
    th[0 * KKp + k] = d->thermo[17 * k + 1];
    for (int c = 0; c < 7; ++c) {
      th[(1 + c) * KKp + k] = d->thermo[17 * k + 3 + c];
      th[(8 + c) * KKp + k] = d->thermo[17 * k + 10 + c];
    }
    wtp[k] = wt[k];
    rwtp[k] = rwt[k];
  }
  std::vector<char> blob;
  auto put = [&](const void* p, size_t bytes) -> int {
    const int off = (int)blob.size();
    blob.insert(blob.end(), (const char*)p, (const char*)p + bytes);
    blob.resize(align16((int)blob.size()), 0);
    return off;
  };
  MechImage& I = m->img;
  I.KK = KK;
  I.KKp = KKp;
  I.sp_one = sp_one;
  I.II = m->II;
  I.IIp = IIp;
  I.G = G;
  I.naux = naux;
  I.o_th = put(th.data(), th.size() * 8);
  I.o_wt = put(wtp.data(), KKp * 8);
  I.o_rwt = put(rwtp.data(), KKp * 8);
  I.o_lnA = put(lnA.data(), IIp * 8);
  I.o_beta = put(beta.data(), IIp * 8);
  I.o_Ea = put(Ea.data(), IIp * 8);
  I.o_rsp = put(urs.data(), IIp * 4);
  I.o_psp = put(ups.data(), IIp * 4);
  I.o_nu = put(unu.data(), IIp * 4);
  I.o_info = put(uinfo.data(), IIp * 4);
  I.o_tb = put(tb.data(), IIp * 4);
  I.o_aux = put(aux.data(), aux.size() * 8);
  I.o_gptr = put(gptr.data(), gptr.size() * 4);
  const int zero = 0;
  const double dzero = 0.0;
  I.o_gsp = gsp.empty() ? put(&zero, 4) : put(gsp.data(), gsp.size() * 4);
  I.o_geff = geff.empty() ? put(&dzero, 8) : put(geff.data(), geff.size() * 8);
  // transposed dense efficiency table geffT[k][17] (64 species rows, stride 17: conflict-free) for
  // the wave kernel (a per-lane walk of the sparse lists measured 0.6 % slower); only for KK <= 63 and
  // G <= 16, and only while the 64-wide launch (12 waves) still fits the 160 KB of LDS with it, else a stub
  const size_t lds_with = blob.size() + 64 * 17 * 8 + 8 * E2T_N + 8 * (size_t)KKp + jscratch_bytes<64>() +
                          12 * (size_t)slice_bytes(G);
  const bool dense = KK <= SP_ONE && G <= 16 && lds_with <= 160 * 1024;
  std::vector<double> geffd(dense ? (size_t)64 * 17 : (size_t)2, 0.0);
  for (int g = 0; dense && g < G; ++g)
    for (int e = gptr[g]; e < gptr[g + 1]; ++e) geffd[(size_t)gsp[e] * 17 + g] = geff[e];
  I.o_geffd = put(geffd.data(), geffd.size() * 8);  // MechView::mgt() tells the two sizes apart
  {
    double e2t[E2T_N];  // 2^(j / E2T_N): E2T_N doubles fill the 64 LDS banks once (conflict-free gathers)
    for (int j = 0; j < E2T_N; ++j) e2t[j] = (double)std::exp2((long double)j / (long double)E2T_N);
    I.o_e2t = put(e2t, sizeof(e2t));
  }
  {
    // element counts of each species for the corrector's element projection, right after e2t (the kernels
    // address it as o_e2t + 8 E2T_N: no extra view field): u64 per species, byte e = the count of the
    // e-th element that occurs in the mechanism (m->npe of them, <= CKMI_PROJ_MMAX; none otherwise)
    std::vector<uint64_t> el(KKp, 0ull);
    m->npe = 0;
    if (d->ncf && d->MM > 0) {
      std::vector<int> used;
      for (int e = 0; e < d->MM; ++e)
        for (int k = 0; k < KK; ++k)
          if (d->ncf[(size_t)e * KK + k] > 0) {
            used.push_back(e);
            break;
          }
      if ((int)used.size() <= CKMI_PROJ_MMAX) {
        m->npe = (int)used.size();
        for (int j = 0; j < m->npe; ++j)
          for (int k = 0; k < KK; ++k)
            el[k] |= (uint64_t)std::min(255, std::max(0, (int)d->ncf[(size_t)used[j] * KK + k])) << (8 * j);
      }
    }
    const int o_el = put(el.data(), el.size() * 8);
    if (o_el != I.o_e2t + 8 * E2T_N) return fail(CKMI_ERR_ARG, "image layout: element table not after e2t");
  }
  I.bytes = (int)blob.size();
  {
    const int* so = nullptr;
    if (upload(m, m->slot_of, &so) != CKMI_OK) return CKMI_ERR_HIP;
    I.slot_of = so;
  }
  {
    // Jacobian column lists of the workgroup kernel (ckmi_big.hip rhs_big): for species j the unit slots
    // naming j, in device-slot order, so that a column block visits only its own slots instead of every
    // slot of every reaction once per block
    std::vector<std::vector<uint32_t>> lists(KK);
    for (int i = 0; i < IIp; ++i) {
      const uint32_t inf = uinfo[i];
      if (inf & RX_GEN) continue;
      const int nr = (inf >> 7) & 7, np = (inf >> 10) & 7;
      for (int sl = 0; sl < 8; ++sl) {
        const bool prod = sl >= 4;
        const int u0 = sl & 3;
        if (u0 >= (prod ? np : nr)) continue;
        const int j = (int)(((prod ? ups[i] : urs[i]) >> (8 * u0)) & 0xffu);
        if (j < KK) lists[j].push_back((uint32_t)i | ((uint32_t)sl << 16));
      }
    }
    std::vector<int> ptr(KK + 1, 0);
    std::vector<uint32_t> ent;
    for (int j = 0; j < KK; ++j) {
      ent.insert(ent.end(), lists[j].begin(), lists[j].end());
      ptr[j + 1] = (int)ent.size();
    }
    if (ent.empty()) ent.push_back(0u);
    const int* dp = nullptr;
    const uint32_t* de = nullptr;
    if (upload(m, ptr, &dp) != CKMI_OK || upload(m, ent, &de) != CKMI_OK) return CKMI_ERR_HIP;
    I.jcol_ptr = dp;
    I.jcol_ent = de;
  }
  void* p = nullptr;
  HIP_CHECK(hipMalloc(&p, blob.size()));
  m->allocs.push_back(p);
  HIP_CHECK(hipMemcpy(p, blob.data(), blob.size(), hipMemcpyHostToDevice));
  I.blob = (const uint4*)p;
  return CKMI_OK;
}

template <int N, bool F64>
size_t reactor_lds_bytes(const ckmi_mech* m) {
  return (size_t)m->img.bytes + jscratch_bytes<N>() + (size_t)rwaves(F64) * slice_bytes(m->G);
}
// Grid = (CUs x resident workgroups per CU), capped by the batch; J workspace = one
// column-major N x 64 matrix per wave slot, allocated stream-ordered (~55 MB for GRI-3.0).
// Per-launch copy of the run configuration: it lives in the launch's stream-ordered workspace,
// so launches with different configurations on one mechanism handle (other streams, other host
// threads) never share it.  The host staging copy is released by a host function enqueued
// behind the copy, i.e. only once the stream has consumed it.
int stage_cfg(const DevCfg& dc, DevCfg* dst, hipStream_t stream) {
  auto* hc = new DevCfg(dc);
  const hipError_t e = hipMemcpyAsync(dst, hc, sizeof(DevCfg), hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) {
    delete hc;
    return fail(CKMI_ERR_HIP, std::string("cfg copy: ") + hipGetErrorString(e));
  }
  HIP_CHECK(hipLaunchHostFunc(stream, [](void* p) { delete static_cast<DevCfg*>(p); }, hc));
  return CKMI_OK;
}

template <int N, bool PL = false, bool F64 = false>
int launch_reactors(const ckmi_mech* m, int n, const DevCfg& dc, const ReactorIO& io, hipStream_t stream,
                    int sel = SEL_ALL) {
  if (!F64 && sel != SEL_NO_PFR) return fail(CKMI_ERR_ARG, "internal: FP32-inverse reactor launch must skip plug flow");
  constexpr int RWAVES = rwaves(F64);
  const size_t lds = reactor_lds_bytes<N, F64>(m);
  static thread_local std::map<int, int> max_lds_set;
  if (lds > 64 * 1024 && max_lds_set[m->device] < (int)lds) {
    HIP_CHECK(hipFuncSetAttribute((const void*)reactor_kernel<N, PL, F64>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
    max_lds_set[m->device] = (int)lds;
  }
  int ncu = 0, per_cu = 0;
  HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, m->device));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, reactor_kernel<N, PL, F64>, RWAVES * WAVE, lds));
  if (per_cu < 1) return fail(CKMI_ERR_SIZE, "reactor kernel does not fit on a CU (LDS " + std::to_string(lds) + " B)");
  const int want = (n + RWAVES - 1) / RWAVES;
  const int grid = std::max(1, std::min(ncu * per_cu, want));
  // the wave's parked Jacobian is FP32 (N x 64 floats per wave slot)
  const size_t jbytes = ((size_t)grid * RWAVES * N * WAVE * sizeof(float) + 255) & ~(size_t)255;
  const size_t cbytes = (sizeof(DevCfg) + 255) & ~(size_t)255;
  void* ws = nullptr;
  HIP_CHECK(hipMallocAsync(&ws, jbytes + cbytes + 256, stream));
  DevCfg* dcfg = (DevCfg*)((char*)ws + jbytes);
  int* queue = (int*)((char*)ws + jbytes + cbytes);
  int rc = stage_cfg(dc, dcfg, stream);
  if (rc == CKMI_OK) {
    HIP_CHECK(hipMemsetAsync(queue, 0, sizeof(int), stream));
    hipLaunchKernelGGL((reactor_kernel<N, PL, F64>), dim3(grid), dim3(RWAVES * WAVE), lds, stream, m->img, dcfg, n, sel,
                       queue, (double*)ws, io);
    HIP_CHECK(hipGetLastError());
  }
  HIP_CHECK(hipFreeAsync(ws, stream));
  return rc;
}

template <int MODE, int NCH, bool PL>
int launch_rop_n(const ckmi_mech* m, int n, const double* T, const double* P, const double* Y, double* o0,
                 double* o1, double* o2, hipStream_t stream) {
  constexpr int NW = rop_waves(NCH);
  const size_t lds = (size_t)m->img.bytes + (size_t)NW * rop_slice_bytes(m->G, m->img.KK, m->img.KKp);
  int ncu = 0, per_cu = 0, lds_max = 0;
  HIP_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, m->device));
  HIP_CHECK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, m->device));
  if (lds > (size_t)lds_max) return fail(CKMI_ERR_SIZE, "mechanism image + ROP work space exceed the LDS of a CU");
  HIP_CHECK(hipFuncSetAttribute((const void*)rop_kernel<MODE, NCH, PL>, hipFuncAttributeMaxDynamicSharedMemorySize,
                                (int)lds));
  HIP_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, rop_kernel<MODE, NCH, PL>, NW * WAVE, lds));
  if (per_cu < 1) return fail(CKMI_ERR_SIZE, "ROP kernel does not fit on a CU");
  const int tasks = (n + ROP_CHUNK - 1) / ROP_CHUNK;
  const int grid = std::max(1, std::min(ncu * per_cu, (tasks + NW - 1) / NW));
  hipLaunchKernelGGL((rop_kernel<MODE, NCH, PL>), dim3(grid), dim3(NW * WAVE), lds, stream, m->img, m->d.orig, n, T, P,
                     Y, o0, o1, o2);
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

template <int MODE>
int launch_rop(const ckmi_mech* m, int n, const double* T, const double* P, const double* Y, double* o0, double* o1,
               double* o2, hipStream_t stream) {
  const bool pl = m->has_plog;
  switch (m->img.KKp / WAVE) {
    case 1: return pl ? launch_rop_n<MODE, 1, true>(m, n, T, P, Y, o0, o1, o2, stream)
                      : launch_rop_n<MODE, 1, false>(m, n, T, P, Y, o0, o1, o2, stream);
    case 2: return pl ? launch_rop_n<MODE, 2, true>(m, n, T, P, Y, o0, o1, o2, stream)
                      : launch_rop_n<MODE, 2, false>(m, n, T, P, Y, o0, o1, o2, stream);
    case 3: return pl ? launch_rop_n<MODE, 3, true>(m, n, T, P, Y, o0, o1, o2, stream)
                      : launch_rop_n<MODE, 3, false>(m, n, T, P, Y, o0, o1, o2, stream);
    case 4: return pl ? launch_rop_n<MODE, 4, true>(m, n, T, P, Y, o0, o1, o2, stream)
                      : launch_rop_n<MODE, 4, false>(m, n, T, P, Y, o0, o1, o2, stream);
    default: return fail(CKMI_ERR_UNSUPPORTED, "mechanism image with more than 255 species");
  }
}

// Makes m's device current for the scope and restores the caller's device afterwards: the
// specialised kernel's module belongs to the device it was loaded on.
struct DeviceScope {
  int prev = -1;
  explicit DeviceScope(int dev) {
    if (hipGetDevice(&prev) != hipSuccess) prev = -1;
    if (prev != dev) (void)hipSetDevice(dev);
  }
  ~DeviceScope() {
    int cur = -1;
    if (prev >= 0 && hipGetDevice(&cur) == hipSuccess && cur != prev) (void)hipSetDevice(prev);
  }
};

// compile and load the specialised ROP kernel of m once (thread-safe), on m's device; CKMI_OK when
// it can run
int jit_ready(ckmi_mech* m) {
  if (!m->jit) return fail(CKMI_ERR_UNSUPPORTED, "no specialised ROP kernel");
  JitRop& J = *m->jit;
  if (J.state.load() == 1) return CKMI_OK;
  std::lock_guard<std::mutex> lk(J.mu);
  if (J.state.load() == 1) return CKMI_OK;
  if (J.state.load() == -1) return fail(CKMI_ERR_UNSUPPORTED, "specialised ROP kernel unavailable: " + J.why);
  std::vector<char> code;
  std::string log;
  const int rc = jit_rop_compile(J.src, code, log);
  if (rc) {
    J.why = "hipRTC compilation failed: " + log.substr(0, 2000);
    J.state.store(-1);
    return fail(CKMI_ERR_HIP, J.why);
  }
  DeviceScope on(m->device);
  if (hipModuleLoadData(&J.mod, code.data()) != hipSuccess ||
      hipModuleGetFunction(&J.fn, J.mod, ("ckjit_rop_k" + std::to_string(m->KK) + "_i" + std::to_string(m->II)).c_str()) !=
          hipSuccess) {
    J.why = "hipModuleLoadData / hipModuleGetFunction failed";
    J.state.store(-1);
    return fail(CKMI_ERR_HIP, J.why);
  }
  J.state.store(1);
  return CKMI_OK;
}

}  // namespace

int ckmi::set_error(int code, const std::string& msg) { return fail(code, msg); }

extern "C" {

const char* ckmi_last_error(void) { return g_err.c_str(); }

#ifdef CKMI_PHASE_TIMERS
// diagnostic build only: buf = device u64 [n][8] (rhs, jac, lu, solve, total cycles)
int ckmi_debug_phase_buffer(void* buf) {
  HIP_CHECK(hipMemcpyToSymbol(HIP_SYMBOL(g_phase_buf), &buf, sizeof(buf)));
  return CKMI_OK;
}
#endif
int ckmi_version(void) { return CKMI_ABI_VERSION; }

int ckmi_mech_create(const ckmi_mech_desc* d, ckmi_mech** out) {
  if (!d || !out) return fail(CKMI_ERR_ARG, "null argument");
  const int KK = d->KK, II = d->II;
  if (KK <= 0 || II < 0) return fail(CKMI_ERR_SIZE, "bad sizes");
  if (KK > KK_IMAGE_MAX) return fail(CKMI_ERR_UNSUPPORTED, "more than 255 species not supported by this build");
  // slot counts and species indices first: everything below (rxn_general, the slot classes, the
  // image) reads [4 i + u] for u < nr[i] / np[i]
  if (const char* bad = ckmi::check_slots(d)) return fail(CKMI_ERR_ARG, bad);
  auto* m = new ckmi_mech();
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) {
    delete m;
    return fail(CKMI_ERR_HIP, "no HIP device");
  }
  m->device = dev;
  m->KK = KK;
  m->II = II;
  {  // runaway guard range from the NASA-7 fits
    double tlo = 1e300, thi = 0.0;
    for (int k = 0; k < KK; ++k) {
      tlo = std::min(tlo, d->thermo[17 * k + 0]);
      thi = std::max(thi, d->thermo[17 * k + 2]);
    }
    m->tguard_lo = 0.5 * tlo;
    m->tguard_hi = 2.0 * thi;  // margin: legitimately hot runs extrapolate the fits (runaways reach 8-10k K)
  }
  // ---- order reactions: elementary, then third-body, then falloff
  std::vector<int> ordr;
  // strips stay type-uniform: chemically activated reactions run in the falloff strips
  // within a type, reactions with at most 2 unit slots per side first: the strips that hold only
  // those skip the slot-2/3 gathers wave-uniformly (eval_rxn_img); general reactions last
  auto slot_class = [&](int i) -> int {
    if (rxn_general(d, i)) return 2;
    double ur = 0.0, up = 0.0;
    for (int u = 0; u < d->nr[i]; ++u) ur += d->rnu[CKMI_SLOTS * i + u];
    for (int u = 0; u < d->np[i]; ++u) up += d->pnu[CKMI_SLOTS * i + u];
    return (ur > 2.0 || up > 2.0) ? 1 : 0;
  };
  std::vector<int> blk(II, -1);  // (rtype, slot class) block of each reaction: lanes swap within one
  for (int t : {CKMI_RXN_ELEMENTARY, CKMI_RXN_LT, CKMI_RXN_THIRDBODY, CKMI_RXN_FALLOFF, CKMI_RXN_CHEMACT, CKMI_RXN_PLOG,
                CKMI_RXN_CHEB})
    for (int cls = 0; cls < 3; ++cls)
      for (int i = 0; i < II; ++i)
        if (d->rtype[i] == t && slot_class(i) == cls) {
          ordr.push_back(i);
          blk[i] = 8 * t + cls;
        }
  for (int i = 0; i < II; ++i) {
    if (d->rtype[i] < 0 || d->rtype[i] > CKMI_RXN_LT) {
      delete m;
      return fail(CKMI_ERR_UNSUPPORTED, "unsupported reaction type");
    }
    if (d->rtype[i] == CKMI_RXN_CHEB) {
      const int p0 = d->plog_ptr ? d->plog_ptr[i] : 0, nrow = d->plog_ptr ? d->plog_ptr[i + 1] - p0 : 0;
      const double* r = d->plog_par ? d->plog_par + 4 * p0 : nullptr;
      const int nt = r && nrow >= 2 ? (int)r[0] : 0, npr = r && nrow >= 2 ? (int)r[1] : 0;
      const bool ok = r && nt >= 1 && nt <= 12 && npr >= 1 && npr <= 12 && nrow == 2 + (nt * npr + 3) / 4 &&
                      r[4] > 0.0 && r[5] > r[4] && r[6] > 0.0 && r[7] > r[6] && !d->has_rev[i];
      if (!ok) {
        delete m;
        return fail(CKMI_ERR_UNSUPPORTED, "Chebyshev record must hold 1..12 x 1..12 coefficients, increasing "
                                          "positive ranges and no REV");
      }
    }
    if (d->rtype[i] == CKMI_RXN_PLOG) {
      const int p0 = d->plog_ptr ? d->plog_ptr[i] : 0, n = d->plog_ptr ? d->plog_ptr[i + 1] - p0 : 0;
      bool ok = d->plog_par && n >= 1 && n <= 64 && !d->has_rev[i];
      for (int j = 0; ok && j + 1 < n; ++j) ok = d->plog_par[4 * (p0 + j)] < d->plog_par[4 * (p0 + j + 1)];
      if (!ok) {
        delete m;
        return fail(CKMI_ERR_UNSUPPORTED, "PLOG table must hold 1..64 points with ascending pressures and no REV");
      }
    }
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
  std::vector<std::array<uint8_t, 8>> perm;
  {
    const char* e = std::getenv("CKMI_LANES");  // A/B knob: CKMI_LANES=0 keeps the file order
    if (e && e[0] == '0') perm.assign(II, {0, 1, 2, 3, 0, 1, 2, 3});
    else assign_lanes(d, slots, blk, perm);
  }
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
    const bool chemact = d->rtype[i] == CKMI_RXN_CHEMACT;  // device type 2 + info bit 13
    const bool cheb = d->rtype[i] == CKMI_RXN_CHEB;        // device type 3 (rate from the aux stream) + bit 15
    const bool lt = d->rtype[i] == CKMI_RXN_LT;            // device type 0 + bit 15 (B, C in the aux record)
    const int type = chemact ? CKMI_RXN_FALLOFF : (cheb ? CKMI_RXN_PLOG : (lt ? CKMI_RXN_ELEMENTARY : d->rtype[i]));
    flags[s] = type | (d->rev[i] ? 4 : 0) | (d->has_rev[i] ? 8 : 0) | ((d->ftype[i] & 7) << 4) | (chemact ? 0x2000 : 0) |
               ((cheb || lt) ? (int)RX_ALT : 0);
    const int nr = d->nr[i], np = d->np[i];
    if (rxn_general(d, i)) {  // FORD / RORD / non-integral: real coefficients, extended variants
      if (type == CKMI_RXN_PLOG || lt) {
        delete m;
        return fail(CKMI_ERR_UNSUPPORTED,
                    "FORD / RORD or non-integral coefficients on a PLOG, Chebyshev or Landau-Teller reaction");
      }
      for (int u = 0; u < nr; ++u)
        if (!(d->rnu[i * CKMI_SLOTS + u] > 0.0) || (d->ford && d->ford[i * CKMI_SLOTS + u] < 0.0)) {
          delete m;
          return fail(CKMI_ERR_UNSUPPORTED, "stoichiometric coefficients must be > 0 and orders >= 0");
        }
      for (int u = 0; u < np; ++u)
        if (!(d->pnu[i * CKMI_SLOTS + u] > 0.0) || (d->rord && d->rord[i * CKMI_SLOTS + u] < 0.0)) {
          delete m;
          return fail(CKMI_ERR_UNSUPPORTED, "stoichiometric coefficients must be > 0 and orders >= 0");
        }
      flags[s] |= RX_GEN;
    }
    if (nr > GEN_SLOTS || np > GEN_SLOTS || ((nr > SLOTS || np > SLOTS) && !(flags[s] & RX_GEN))) {
      delete m;
      return fail(CKMI_ERR_UNSUPPORTED, "more than 8 species on a reaction side");
    }
    nrp[s] = nr | (np << 8);
    int rr[4] = {0, 0, 0, 0}, pp[4] = {0, 0, 0, 0};
    double sf = 0.0, sr = 0.0;
    // per-slot device arrays hold the first SLOTS species (a general reaction reads its aux stream)
    for (int u = 0; u < nr; ++u) {
      if (u < SLOTS) {
        rr[u] = d->rsp[i * CKMI_SLOTS + u];
        rnu[u * IIpad + s] = d->rnu[i * CKMI_SLOTS + u];
      }
      sf += d->rnu[i * CKMI_SLOTS + u];
    }
    for (int u = 0; u < np; ++u) {
      if (u < SLOTS) {
        pp[u] = d->psp[i * CKMI_SLOTS + u];
        pnu[u * IIpad + s] = d->pnu[i * CKMI_SLOTS + u];
      }
      sr += d->pnu[i * CKMI_SLOTS + u];
    }
    rsp[s] = make_int4(rr[0], rr[1], rr[2], rr[3]);
    psp[s] = make_int4(pp[0], pp[1], pp[2], pp[3]);
    dnu[s] = sr - sf;
    ordf[s] = sf;
    ordrr[s] = sr;
    const bool plog = type == CKMI_RXN_PLOG;  // PLOG / CHEB: rate from the aux stream; the slot holds ln 1, 0, 0
    lnA[s] = plog ? 0.0 : d->arr[3 * i];
    beta[s] = plog ? 0.0 : d->arr[3 * i + 1];
    Ea[s] = plog ? 0.0 : d->arr[3 * i + 2];
    lnA0[s] = d->low[3 * i];
    beta0[s] = d->low[3 * i + 1];
    Ea0[s] = d->low[3 * i + 2];
    for (int c = 0; c < 5; ++c) fp[c * IIpad + s] = d->fpar[5 * i + c];
    rlnA[s] = d->revp[3 * i];
    rbeta[s] = d->revp[3 * i + 1];
    rEa[s] = d->revp[3 * i + 2];
    if (type == 1 || type == 2) tb[s] = d->tbsp[i] >= 0 ? -(d->tbsp[i] + 2) : group_of(i);
  }
  m->G = (int)gmap.size();
  m->rtype_orig.assign(d->rtype, d->rtype + II);
  // PLOG and chemically activated reactions are evaluated by the extended kernel variant
  m->has_plog = std::count(d->rtype, d->rtype + II, (int32_t)CKMI_RXN_PLOG) > 0 ||
                std::count(d->rtype, d->rtype + II, (int32_t)CKMI_RXN_CHEMACT) > 0 ||
                std::count(d->rtype, d->rtype + II, (int32_t)CKMI_RXN_CHEB) > 0 ||
                std::count(d->rtype, d->rtype + II, (int32_t)CKMI_RXN_LT) > 0;
  for (int i = 0; i < II; ++i) m->has_general = m->has_general || rxn_general(d, i);
  m->has_plog = m->has_plog || m->has_general;
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
  rc |= build_image(m, d, slots, flags, nrp, rsp, psp, rnu, pnu, lnA, beta, Ea, lnA0, beta0, Ea0, fp, rlnA, rbeta, rEa,
                    tb, gptr, gsp, geff, wt, rwt, perm);
  if (rc) {
    ckmi_mech_destroy(m);
    return rc;
  }
  // the mechanism-specialised ROP kernel: source and parameter block now, compilation at first use
  m->jit = new JitRop();
  {
    std::vector<double> prm;
    const char* env = std::getenv("CKMI_ROP_JIT");
    if (env && env[0] == '0') {
      m->jit->state = -1;
      m->jit->why = "disabled by CKMI_ROP_JIT=0";
    } else if (!jit_rop_generate(d, m->jit->src, prm, m->jit->lnA_off, m->jit->why)) {
      m->jit->state = -1;
    } else {
      const double* p = nullptr;
      if (upload(m, prm, &p)) {
        ckmi_mech_destroy(m);
        return CKMI_ERR_HIP;
      }
      m->jit->prm = const_cast<double*>(p);
      if (const char* dump = std::getenv("CKMI_JIT_DUMP")) {
        if (FILE* f = std::fopen(dump, "w")) {
          std::fputs(m->jit->src.c_str(), f);
          std::fclose(f);
        }
      }
    }
  }
  *out = m;
  return CKMI_OK;
}

int ckmi_mech_destroy(ckmi_mech* m) {
  if (!m) return CKMI_OK;
  if (m->jit) {
    if (m->jit->mod) (void)hipModuleUnload(m->jit->mod);
    delete m->jit;
  }
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
  if (m->rtype_orig[irxn] == CKMI_RXN_PLOG || m->rtype_orig[irxn] == CKMI_RXN_CHEB)
    return fail(CKMI_ERR_UNSUPPORTED, "A-factor of a PLOG / Chebyshev reaction (its rate comes from its table)");
  const double lnA = std::log(A);
  m->lnA_orig[irxn] = lnA;
  const int s = m->slot_of[irxn];
  HIP_CHECK(hipMemcpy(const_cast<double*>(m->d.lnA) + s, &lnA, sizeof(double), hipMemcpyHostToDevice));
  HIP_CHECK(hipMemcpy((char*)m->img.blob + m->img.o_lnA + sizeof(double) * s, &lnA, sizeof(double),
                      hipMemcpyHostToDevice));
  if (m->jit && m->jit->prm) {
    HIP_CHECK(hipMemcpy(m->jit->prm + m->jit->lnA_off[irxn], &lnA, sizeof(double), hipMemcpyHostToDevice));
    if (m->b_orig[irxn] == 0.0 && m->E_orig[irxn] == 0.0)  // k = A reactions read A itself (ckmi_jit.cpp)
      HIP_CHECK(hipMemcpy(m->jit->prm + m->jit->lnA_off[irxn] + 1, &A, sizeof(double), hipMemcpyHostToDevice));
  }
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
  const int path = g_rop_path.load();
  if (path == 2 || (path == 0 && n >= JIT_MIN_STATES)) {
    const int rc = jit_ready(const_cast<ckmi_mech*>(m));
    if (rc == CKMI_OK) {
      DeviceScope on(m->device);
      void* args[] = {&n, (void*)&T, (void*)&P, (void*)&Y, &wdot, &cp, &h, &m->jit->prm};
      HIP_CHECK(hipModuleLaunchKernel(m->jit->fn, (unsigned)((n + 63) / 64), 1, 1, 64, 1, 1, 0, (hipStream_t)stream,
                                      args, nullptr));
      return CKMI_OK;
    }
    if (path == 2) return rc;
  }
  return launch_rop<0>(m, n, T, P, Y, wdot, cp, h, (hipStream_t)stream);
}

int ckmi_set_rop_path(int32_t path) {
  if (path < 0 || path > 2) return fail(CKMI_ERR_ARG, "rop path must be 0 (auto), 1 (generic) or 2 (specialised)");
  g_rop_path = path;
  return CKMI_OK;
}

int ckmi_rop_jit_source(const ckmi_mech_desc* d, char* buf, int64_t cap, int64_t* len) {
  if (!d || !len) return fail(CKMI_ERR_ARG, "null argument");
  std::string src, why;
  std::vector<double> prm;
  std::vector<int> off;
  if (!jit_rop_generate(d, src, prm, off, why)) return fail(CKMI_ERR_UNSUPPORTED, why);
  *len = (int64_t)src.size();
  if (buf && cap > 0) {
    const size_t k = std::min<size_t>((size_t)cap - 1, src.size());
    std::memcpy(buf, src.data(), k);
    buf[k] = 0;
  }
  return CKMI_OK;
}

int ckmi_rop_jit_compile(const ckmi_mech_desc* d, int64_t* code_bytes) {
  if (!d || !code_bytes) return fail(CKMI_ERR_ARG, "null argument");
  std::string src, why, log;
  std::vector<double> prm;
  std::vector<int> off;
  if (!jit_rop_generate(d, src, prm, off, why)) return fail(CKMI_ERR_UNSUPPORTED, why);
  std::vector<char> code;
  if (jit_rop_compile(src, code, log)) return fail(CKMI_ERR_HIP, "hipRTC compilation failed: " + log.substr(0, 2000));
  *code_bytes = (int64_t)code.size();
  return CKMI_OK;
}

int ckmi_rop_jit_state(const ckmi_mech* m, int32_t* state) {
  if (!m || !state) return fail(CKMI_ERR_ARG, "null argument");
  *state = m->jit ? m->jit->state.load() : -1;
  if (*state == -1 && m->jit) {
    std::lock_guard<std::mutex> lk(m->jit->mu);
    g_err = m->jit->why;
  }
  return CKMI_OK;
}

int ckmi_reaction_rates(const ckmi_mech* m, int32_t n, const double* T, const double* P, const double* Y, double* qf,
                        double* qr, void* stream) {
  if (!m || n < 0 || !qf || !qr) return fail(CKMI_ERR_ARG, "bad argument");
  if (n == 0) return CKMI_OK;
  return launch_rop<1>(m, n, T, P, Y, qf, qr, nullptr, (hipStream_t)stream);
}

int ckmi_reactor_run_ex(const ckmi_mech* m, const ckmi_reactor_cfg* cfg, int32_t n, const int32_t* problem,
                        const double* T0, const double* P0, const double* V0, const double* Y0,
                        const ckmi_reactor_ext* ext, double* tau, double* Tend, double* Pend, double* Vend,
                        double* Yend, int32_t* stats, int32_t nsave, const double* t_save, double* y_save,
                        void* stream) {
  if (!m || !cfg || n < 0) return fail(CKMI_ERR_ARG, "bad argument");
  if (cfg->nprof < 0 || cfg->nprof > 64) return fail(CKMI_ERR_ARG, "nprof must be in [0, 64]");
  if (!(cfg->t_end > 0.0) || !(cfg->rtol > 0.0) || !(cfg->atol > 0.0)) return fail(CKMI_ERR_ARG, "t_end, rtol, atol must be > 0");
  if (cfg->energy != 1 && cfg->energy != 2) return fail(CKMI_ERR_ARG, "energy must be 1 or 2");
  if (cfg->ign_mode < 0 || cfg->ign_mode > 4) return fail(CKMI_ERR_ARG, "bad ignition mode");
  if (cfg->ign_mode == 4 && (cfg->ign_species < 0 || cfg->ign_species >= m->KK)) return fail(CKMI_ERR_ARG, "bad KLIM species");
  if (cfg->prof_kind != 0 && cfg->prof_kind != 1) return fail(CKMI_ERR_ARG, "prof_kind must be 0 (VPRO/PPRO) or 1 (TPRO)");
  if (cfg->prof_kind == 1 && cfg->energy != 2) return fail(CKMI_ERR_ARG, "TPRO needs a given-temperature run (energy = 2)");
  if (!(cfg->gfac >= 0.0)) return fail(CKMI_ERR_ARG, "GFAC must be >= 0");
  if (!(cfg->htc >= 0.0) || !(cfg->areaq >= 0.0) || !(cfg->tamb > 0.0 || cfg->htc * cfg->areaq == 0.0))
    return fail(CKMI_ERR_ARG, "HTC, AREAQ must be >= 0 and TAMB > 0");
  if (cfg->asteps < 0) return fail(CKMI_ERR_ARG, "asteps must be >= 0");
  if (nsave > 0 && (!t_save || !y_save)) return fail(CKMI_ERR_ARG, "t_save / y_save required when nsave > 0");
  if (ext && (ext->afac_rxn != nullptr) != (ext->afac != nullptr)) return fail(CKMI_ERR_ARG, "afac_rxn and afac go together");
  if (ext && ext->n_adap && (ext->max_adap <= 0 || !ext->t_adap || !ext->y_adap))
    return fail(CKMI_ERR_ARG, "n_adap needs max_adap > 0, t_adap and y_adap");
  if (cfg->nprof2 < 0 || cfg->nprof2 > 64) return fail(CKMI_ERR_ARG, "nprof2 must be in [0, 64]");
  if (cfg->nprof2 > 0 && cfg->prof2_kind != 1 && cfg->prof2_kind != 2)
    return fail(CKMI_ERR_ARG, "prof2_kind must be 1 (QPRO) or 2 (AEXT)");
  if (cfg->nprof2 > 0 && cfg->energy != 1) return fail(CKMI_ERR_ARG, "QPRO / AEXT need an energy-equation run");
  if (cfg->nprof3 < 0 || cfg->nprof3 > 64) return fail(CKMI_ERR_ARG, "nprof3 must be in [0, 64]");
  if (cfg->nprof3 > 0 && !(cfg->nprof2 > 0 && cfg->prof2_kind == 1))
    return fail(CKMI_ERR_ARG, "the third profile (AEXT) needs a QPRO second profile");
  if (cfg->avar > m->KK || cfg->avar < -1) return fail(CKMI_ERR_ARG, "avar must be -1, 0 (T) or 1 + species index");
  if (cfg->eng[CKMI_ENG_HTMODEL] == 1.0 && !cfg->tran)
    return fail(CKMI_ERR_ARG, "the engine's ICHX heat transfer needs the transport fits (cfg->tran)");
  if (n == 0) return CKMI_OK;
  DevCfg dc;  // this call's configuration (staged per launch: no state shared between calls)
  {
    dc.c = *cfg;
    if (dc.c.gfac == 0.0) dc.c.gfac = 1.0;
    std::vector<double> tc;
    for (int i = 0; i < cfg->nprof; ++i)
      if (cfg->prof_t[i] > 0.0 && cfg->prof_t[i] < cfg->t_end) tc.push_back(cfg->prof_t[i]);
    for (int i = 0; i < cfg->nprof2; ++i)
      if (cfg->prof2_t[i] > 0.0 && cfg->prof2_t[i] < cfg->t_end) tc.push_back(cfg->prof2_t[i]);
    for (int i = 0; i < cfg->nprof3; ++i)
      if (cfg->prof3_t[i] > 0.0 && cfg->prof3_t[i] < cfg->t_end) tc.push_back(cfg->prof3_t[i]);
    std::sort(tc.begin(), tc.end());
    tc.erase(std::unique(tc.begin(), tc.end()), tc.end());
    dc.ncrit = (int)tc.size();
    std::copy(tc.begin(), tc.end(), dc.tcrit);
    dc.guard_y = std::max(1e-3, 1e3 * cfg->atol);
    dc.guard_tlo = m->tguard_lo;
    dc.guard_thi = m->tguard_hi;
    dc.npe = cfg->no_elem_proj ? 0 : m->npe;
  }
  ReactorIO io{problem, T0, P0, V0, Y0, tau, Tend, Pend, Vend, Yend, stats, nsave, t_save, y_save,
               ext ? ext->afac_rxn : nullptr, ext ? ext->afac : nullptr, ext ? ext->max_adap : 0,
               ext ? ext->t_adap : nullptr, ext ? ext->y_adap : nullptr, ext ? ext->n_adap : nullptr,
               ext ? ext->t_stop : nullptr};
  const int nvar = m->KK + 1;
  int rc;
  // PLOG mechanisms use one (64-wide) reactor variant, so that the PLOG branch costs compile time once
  // more than 63 species: one workgroup per reactor (ckmi_big.hip); else one wave per reactor, its
  // Newton inverse stored in FP64 when the tolerances ask for more than its FP32 rounding resolves
  // (rtol < 1e-9; measured: the FP32-stored inverse integrates the rtol = 1e-8 sweeps of configs[2]
  // and [3] without a failure, and fails one of 55 reactors at rtol = 1e-10, atol = 1e-20), and for
  // mechanisms with FORD / RORD / fractional orders, whose d C^o / dC = o C^(o-1) grows without
  // bound as C -> 0 (the FP32-stored inverse of such a Newton matrix stalled one reactor of five)
  const int rpath = g_reactor_path.load();
  const bool f64 = rpath == 2 || (rpath != 3 && (cfg->rtol < 1e-9 || m->has_general));
  const hipStream_t st = (hipStream_t)stream;
  // An FP32-inverse launch skips the plug-flow reactors and an FP64-inverse launch of the same size
  // follows it for them (it pulls and drops the other indices: ~0.1 ms per 65,536 reactors when
  // there are none); the problem array is device memory, so the host cannot tell in advance.
  const int no_pf = SEL_NO_PFR;
  if (nvar > 64 || rpath == 1) {
    // the workgroup kernel has no engine model: checked on the host (one synchronous copy of problem[])
    std::vector<int32_t> hp(n);
    HIP_CHECK(hipMemcpyAsync(hp.data(), problem, sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
    HIP_CHECK(hipStreamSynchronize(st));
    if (std::find(hp.begin(), hp.end(), 4) != hp.end())
      return fail(CKMI_ERR_UNSUPPORTED, "engine reactors (problem 4) need KK + 1 <= 64 (the wave-per-reactor kernel)");
    rc = launch_big_reactors(m, n, dc, io, st);
  }
#ifdef CKMI_PROBE_C3
  // ISA probe build (scripts/isa_probe.sh): only the configs[2] kernel is instantiated, so that its
  // register / scratch figures come out of a one-variant compile; never linked into libckmi.so
  else rc = launch_reactors<54>(m, n, dc, io, st, no_pf);
#else
  else if (m->has_plog) {
    rc = f64 ? launch_reactors<64, true, true>(m, n, dc, io, st) : launch_reactors<64, true>(m, n, dc, io, st, no_pf);
    if (!rc && !f64) rc = launch_reactors<64, true, true>(m, n, dc, io, st, SEL_PFR);
  } else if (nvar <= 54) {
    if (f64) rc = launch_reactors<54, false, true>(m, n, dc, io, st);
    else {
      rc = nvar <= 32 ? launch_reactors<32>(m, n, dc, io, st, no_pf) : launch_reactors<54>(m, n, dc, io, st, no_pf);
      if (!rc) rc = launch_reactors<54, false, true>(m, n, dc, io, st, SEL_PFR);
    }
  } else {
    rc = f64 ? launch_reactors<64, false, true>(m, n, dc, io, st) : launch_reactors<64>(m, n, dc, io, st, no_pf);
    if (!rc && !f64) rc = launch_reactors<64, false, true>(m, n, dc, io, st, SEL_PFR);
  }
#endif
  if (rc) return rc;
  HIP_CHECK(hipGetLastError());
  return CKMI_OK;
}

int ckmi_engine_heat_rates(const ckmi_mech* m, const ckmi_reactor_cfg* cfg, double T0, double P0, const double* Y0,
                           int32_t n, const double* t, const double* y, double* ahrr, double* qloss, void* stream) {
  if (!m || !cfg || n < 0 || !Y0 || (n > 0 && (!t || !y || !ahrr || !qloss))) return fail(CKMI_ERR_ARG, "bad argument");
  if (!(T0 > 0.0) || !(P0 > 0.0)) return fail(CKMI_ERR_ARG, "T0 and P0 must be > 0");
  if (m->KK + 1 > WAVE) return fail(CKMI_ERR_UNSUPPORTED, "engine heat rates need KK + 1 <= 64 (as engine runs)");
  if (cfg->eng[CKMI_ENG_HTMODEL] == 1.0 && !cfg->tran)
    return fail(CKMI_ERR_ARG, "the engine's ICHX heat transfer needs the transport fits (cfg->tran)");
  if (n == 0) return CKMI_OK;
  DevCfg dc;
  dc.c = *cfg;
  if (dc.c.gfac == 0.0) dc.c.gfac = 1.0;
  dc.ncrit = 0;
  dc.guard_y = std::max(1e-3, 1e3 * cfg->atol);
  dc.guard_tlo = m->tguard_lo;
  dc.guard_thi = m->tguard_hi;
  dc.npe = 0;  // (no integration)
  const hipStream_t st = (hipStream_t)stream;
  const size_t lds = (size_t)align16(m->img.bytes) + slice_vec_bytes(m->G) + align16((int)sizeof(RunCtx));
  const void* fn = m->has_plog ? (const void*)engine_heat_kernel<true> : (const void*)engine_heat_kernel<false>;
  if (lds > 64 * 1024) HIP_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  const size_t cbytes = (sizeof(DevCfg) + 255) & ~(size_t)255;
  void* ws = nullptr;
  HIP_CHECK(hipMallocAsync(&ws, cbytes, st));
  int rc = stage_cfg(dc, (DevCfg*)ws, st);
  if (rc == CKMI_OK) {
    const int grid = std::min(n, 4096);
    if (m->has_plog)
      hipLaunchKernelGGL(engine_heat_kernel<true>, dim3(grid), dim3(WAVE), lds, st, m->img, (const DevCfg*)ws, T0, P0,
                         Y0, n, t, y, ahrr, qloss);
    else
      hipLaunchKernelGGL(engine_heat_kernel<false>, dim3(grid), dim3(WAVE), lds, st, m->img, (const DevCfg*)ws, T0, P0,
                         Y0, n, t, y, ahrr, qloss);
    HIP_CHECK(hipGetLastError());
  }
  HIP_CHECK(hipFreeAsync(ws, st));
  return rc;
}

int ckmi_set_reactor_path(int32_t path) {
  if (path < 0 || path > 3)
    return fail(CKMI_ERR_ARG, "reactor path must be 0 (automatic), 1 (workgroup), 2 (wave, FP64 inverse) or 3 (wave, "
                              "FP32-stored inverse)");
  g_reactor_path = path;
  return CKMI_OK;
}

int ckmi_reactor_run(const ckmi_mech* m, const ckmi_reactor_cfg* cfg, int32_t n, const int32_t* problem,
                     const double* T0, const double* P0, const double* V0, const double* Y0, double* tau, double* Tend,
                     double* Pend, double* Vend, double* Yend, int32_t* stats, int32_t nsave, const double* t_save,
                     double* y_save, void* stream) {
  return ckmi_reactor_run_ex(m, cfg, n, problem, T0, P0, V0, Y0, nullptr, tau, Tend, Pend, Vend, Yend, stats, nsave,
                             t_save, y_save, stream);
}

}  // extern "C"
