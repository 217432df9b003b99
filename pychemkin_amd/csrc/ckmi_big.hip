// ckmi_big.hip -- batch reactors of mechanisms with more than 63 species (64 <= KK + 1 <= 192):
// one workgroup of 4 waves integrates one reactor (SURVEY.md §8(d) configs[4]: ~160 species).
//
// The wave-per-reactor kernel of ckmi.hip keeps the whole Newton matrix (n <= 64) in one wave's
// registers.  A 162 x 162 matrix (207 KB in FP64) fits neither one wave nor the 160 KB LDS of a CU,
// but it fits the register file of a whole CU: the workgroup is four waves (one per SIMD, so each
// wave may address the unified 512-register file, VGPRs + AGPRs) and thread i owns
//   * state component i (0 = T, 1 + k = Y_k) of every integrator vector, and
//   * row i of the Newton matrix, NC doubles in registers (NC = n rounded up to 16, identity
//     padding), inverted in place by Gauss-Jordan with partial pivoting.  The pivot column is
//     kept at register 0: every elimination step shifts the row by one register while it
//     updates it (a[m-1] = a[m] - g p[m]), so the pivot loop is a run-time loop over an
//     unrolled, statically indexed row update; after NC steps the columns are back in order.
// A Newton solve is then one matrix-vector product (no triangular dependency chains).
//
// The integrator is the same CVODE-style BDF state machine as ckmi.hip (control flow identical to
// oracle/ckoracle.c).  Its scalar state is replicated: each wave keeps its own copy in LDS and
// runs the same control code; every decision is taken on workgroup reductions (DPP inside a wave,
// LDS + s_barrier across the four) whose results are bitwise identical in every wave, so the copies
// never diverge and all waves pass the same barriers.
//
// Right-hand side: species thermo with thread = species, the reactions in 64-reaction strips over
// the four waves; each wave accumulates wdot (and dwdot/dT) into a private LDS copy that is summed
// in a fixed order -- results are deterministic, independent of wave timing.  Jacobian (rare: ~2 %
// of the RHS calls): the reaction pass stores dq/dC of every slot in a per-workgroup HBM buffer;
// J is then assembled column block by column block in LDS (each wave owns a quarter of the block's
// columns, so every LDS atomic target is written by one wave only), its energy row is formed, and
// the block is parked in FP32 in the workgroup's HBM slot (M = I - gamma J is rebuilt from it at
// every setup; the oracle rounds J the same way).
#include <hip/hip_runtime.h>

#include <type_traits>

#include <algorithm>
#include <climits>
#include <cmath>
#include <map>
#include <string>

#include "ckmi_internal.hpp"
#include "ckmi_run.hpp"

namespace ckmi {
namespace {

constexpr int BW = 4;           // waves per workgroup
constexpr int NT = BW * WAVE;   // threads: state component / matrix row per thread
constexpr int BIG_NMAX = 192;   // n = KK + 1 <= 192
constexpr int RED_SET = 72;     // doubles per reduction set (two sets alternate): [BW][16] + [BW] for bsumn_max<16>
constexpr int NDQ = 16;         // dq/dC slots per reaction: unit reactions 4 + 4, general ones GEN_SLOTS + GEN_SLOTS
constexpr int XS = NT + 16;     // row stride of the MFMA form's solve partial sums [NB][XS] (bank-conflict-free)
// q-block stride of a wave's diagonal-block buffer [4 q][16 ti][NB c] (BigMatrixM::blk_buf): 8 mod 32
// doubles, so the A-operand reads of the four q blocks fall in disjoint bank ranges
constexpr int big_qb(int NB) { return 16 * NB + ((8 - (16 * NB) % 32) + 32) % 32; }

// Diagnostic build only (-DCKMI_PHASE_TIMERS, scripts/phase_profile.py --big): per-reactor shader
// cycles per phase into a debug buffer [n][16]: rhs, rhs+J, build, factor, solve, total, then the
// factorisation split of wave 0 (MFMA form: own panels, barrier, -, pivot-row gather, MFMA, restore).
#ifdef CKMI_PHASE_TIMERS
__device__ unsigned long long* g_big_phase_buf = nullptr;
#define BPH_T0() const unsigned long long _bph0 = __builtin_amdgcn_s_memtime()
#define BPH_ADD(slot) bph[slot] += __builtin_amdgcn_s_memtime() - _bph0
#else
#define BPH_T0() (void)0
#define BPH_ADD(slot) (void)0
#endif

#define BIG_CHECK(x)                                                                                 \
  do {                                                                                              \
    hipError_t _e = (x);                                                                            \
    if (_e != hipSuccess) return set_error(CKMI_ERR_HIP, std::string(#x) + ": " + hipGetErrorString(_e)); \
  } while (0)

// LDS layout of the workgroup (byte offsets; the mechanism image is at 0)
struct BigLds {
  int C, gRT, hRT, ek;   // [KKp] species vectors
  int wdot, dwdT;        // [BW][KKp] per-wave accumulators
  int Mg;                // [G]
  int zn;                // [QMAX + 1][NT] Nordsieck history
  int prow;              // [BW][4][NBP] per-wave pivot-row entries
  int gcol;              // [2][16][NBP] raw pivot column (per ti), double-buffered by step parity
  int phdr;              // [2] PivHdr
  int perm, rank;        // int [NT] pivot row of step k / step of row i
  int bp;                // [NT] permuted right-hand side
  int xpart;             // partial row sums of a solve, [NT][NBP] (BigMatrix) or [NB][XS] (BigMatrixM); aliases
                         // the Jacobian block
  int red;               // [2][RED_SET] reduction sets
  int ctl;               // [BW] per-wave control copies (BdfS, Ctl, Ign, RunCtx)
  int jblk;              // [jcb][LDJ] Jacobian column block
  int jcb;               // columns per block (multiple of BW)
  int bytes;
};
constexpr int CTL_BYTES = align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) + align16((int)sizeof(Ign)) +
                          align16((int)sizeof(RunCtx));

// ------------------------------------------------------------------ workgroup reductions
// All threads call these at the same program points.  Each flips the set it uses, so a wave
// that races ahead to the next reduction cannot overwrite a set another wave is still reading
// (it would first have to pass the barrier of the reduction in between).
struct Blk {
  int ored;
  int phase;
  __device__ __forceinline__ double* set() const { return lds_at<double>(ored) + phase * RED_SET; }
};

__device__ __forceinline__ double bsum(Blk& B, double v, int wid, int lane) {
  const double w = wave_sum(v);
  double* r = B.set();
  if (lane == 0) r[wid] = w;
  __syncthreads();
  const double s = (r[0] + r[1]) + (r[2] + r[3]);
  B.phase ^= 1;
  return s;
}
__device__ __forceinline__ void bsum2(Blk& B, double& a, double& b, int wid, int lane) {
  const double wa = wave_sum(a), wb = wave_sum(b);
  double* r = B.set();
  if (lane == 0) {
    r[wid] = wa;
    r[4 + wid] = wb;
  }
  __syncthreads();
  a = (r[0] + r[1]) + (r[2] + r[3]);
  b = (r[4] + r[5]) + (r[6] + r[7]);
  B.phase ^= 1;
}
// sum of v over the workgroup, and x of thread src broadcast, in one barrier
__device__ __forceinline__ double bsum_bcast(Blk& B, double v, double& x, int src, int tid, int wid, int lane) {
  const double w = wave_sum(v);
  double* r = B.set();
  if (lane == 0) r[wid] = w;
  if (tid == src) r[8] = x;
  __syncthreads();
  const double s = (r[0] + r[1]) + (r[2] + r[3]);
  x = r[8];
  B.phase ^= 1;
  return s;
}
__device__ __forceinline__ double bbcast(Blk& B, double x, int src, int tid) {
  double* r = B.set();
  if (tid == src) r[8] = x;
  __syncthreads();
  x = r[8];
  B.phase ^= 1;
  return x;
}
__device__ __forceinline__ int bbcast_int(Blk& B, int x, int src, int tid) {
  int* r = reinterpret_cast<int*>(B.set());
  if (tid == src) r[0] = x;
  __syncthreads();
  x = r[0];
  B.phase ^= 1;
  return x;
}
__device__ __forceinline__ double bmax(Blk& B, double v, int wid, int lane) {
  const double w = wave_max(v);
  double* r = B.set();
  if (lane == 0) r[wid] = w;
  __syncthreads();
  const double s = fmax(fmax(r[0], r[1]), fmax(r[2], r[3]));
  B.phase ^= 1;
  return s;
}
// NV (<= 8) sums over the workgroup in one barrier: each wave's multi-value reduction (wave_sum_multi's
// stages), the lanes holding a value publish it, every thread adds the four wave partials in a fixed order
template <int NV>
__device__ __forceinline__ void bsumn(Blk& B, double (&v)[NV], int wid, int lane) {
  static_assert(NV * BW <= RED_SET, "reduction set too small");
  wave_sum_stages<0, NV>(v, lane);
  double* r = B.set();
  if ((lane & (64 / NV - 1)) == 0) r[wid * NV + wave_sum_index<NV>(lane)] = v[0];
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = (r[j] + r[NV + j]) + (r[2 * NV + j] + r[3 * NV + j]);
  B.phase ^= 1;
}
__device__ __forceinline__ void bsum8(Blk& B, double (&v)[8], int wid, int lane) { bsumn<8>(B, v, wid, lane); }
// bsumn and the workgroup maximum of mx, in the same barrier
template <int NV>
__device__ __forceinline__ void bsumn_max(Blk& B, double (&v)[NV], double& mx, int wid, int lane) {
  static_assert(NV * BW + BW <= RED_SET, "reduction set too small");
  wave_sum_stages<0, NV>(v, lane);
  const double wm = wave_max(mx);
  double* r = B.set();
  if ((lane & (64 / NV - 1)) == 0) r[wid * NV + wave_sum_index<NV>(lane)] = v[0];
  if (lane == 0) r[BW * NV + wid] = wm;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < NV; ++j) v[j] = (r[j] + r[NV + j]) + (r[2 * NV + j] + r[3 * NV + j]);
  mx = fmax(fmax(r[BW * NV], r[BW * NV + 1]), fmax(r[BW * NV + 2], r[BW * NV + 3]));
  B.phase ^= 1;
}
__device__ __forceinline__ double bwrms(Blk& B, double v, double ewt, int n, int wid, int lane) {
  const double x = v * ewt;
  return sqrt(bsum(B, x * x, wid, lane) / n);
}

// ------------------------------------------------------------------ element projection
// The workgroup form of elem_project_wave (ckmi_reactor.hpp; oracle elem_project): thread = component.  The
// element sums r[e] = sum_k C_ek y_k come from the step's fused reduction (ST_STEP_COMPLETE); past the
// threshold (rare) the Gram matrix by bsum8 batches and the solve by thread 0 in the scratch scr, read back
// after a barrier.  Every wave takes the same decision from the same sums.
__device__ __forceinline__ void elem_project_big(const MechView& V, Blk& B, int npe, const double (&r)[PROJ_MMAX],
                                                 const double* eb0, double rtol, double y, double& acor, int tid,
                                                 int wid, int lane, double* scr) {
  double v[PROJ_MMAX];
  double rmax = 0.0, bmax = 0.0;
#pragma unroll
  for (int e = 0; e < PROJ_MMAX; ++e) {
    v[e] = 0.0;
    if (e < npe) {
      v[e] = r[e] - eb0[e];
      rmax = fmax(rmax, fabs(v[e]));
      bmax = fmax(bmax, eb0[e]);
    }
  }
  if (!(rmax > PROJ_TOL * rtol * bmax)) return;
  const bool isp = tid >= 1 && tid <= V.KK;
  const int s = isp ? tid - 1 : 0;
  const uint64_t cnt = isp ? elem_table(V)[s] : 0ull;
  const double rw = isp ? V.rwt()[s] : 0.0;
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
    bsum8(B, g, wid, lane);
    if (tid == 0) {
#pragma unroll
      for (int i = 0; i < 8; ++i)
        if (p0 + i < npair) scr[p0 + i] = g[i];
    }
  }
  if (tid == 0) {
#pragma unroll
    for (int e = 0; e < PROJ_MMAX; ++e) {
      if (e < npe) {
        scr[PROJ_SCR_RES + e] = v[e];
        if (!(eb0[e] > PROJ_TRACE * bmax)) scr[e * (e + 1) / 2 + e] = 0.0;  // trace element: left out
      }
    }
    proj_solve_lds(scr, npe);
  }
  __syncthreads();
  double sc = 0.0;
#pragma unroll
  for (int e = 0; e < PROJ_MMAX; ++e)
    if (e < npe) sc += elem_coef(cnt, rw, e) * scr[PROJ_SCR_LAM + e];
  acor -= w * sc;
  __syncthreads();  // scr is free again (the next projection's thread 0 may not overwrite it earlier)
}

#include "ckmi_big_matrix.hpp"

// ------------------------------------------------------------------ general reactions
// FORD / RORD orders and non-integral coefficients (mechanisms flagged has_general, PL = true):
// the reaction keeps no unit slots, its species, coefficients and orders are in the aux stream
// (eval_gen_img).  RHS: q scattered with the real coefficients into this wave's wdot copy; with
// the Jacobian, dwdot/dT through the orders and dq/dC of each slot (the chord rule of dconc_pow)
// into the reaction's Dg slots (reactants 0..GEN_SLOTS-1, products GEN_SLOTS..), as oracle reactor_rhs.
__device__ __noinline__ void gen_rhs_big(const MechView& V, const RunCtx& R, int i, uint32_t inf, double T,
                                         double lnT, double invT, double lnPRT, double P, const double* C,
                                         const double* gRT, const double* hRT, const double* Mg, double* wdw,
                                         double* dwdw, int conp, bool with_j, double* __restrict__ Dg, int IIp) {
  const double* g;
  const Rxn e = eval_gen_img(V, i, inf, T, lnT, invT, lnPRT, P, C, gRT, hRT, Mg, with_j, R.pslot, R.plnf, R.gfac, g);
  const double* e2t = V.e2t();
  const int nr = (int)g[0], np = (int)g[1];
  const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
  for (int u = 0; u < nr; ++u) atomicAdd(&wdw[(int)g[2 + 3 * u]], -g[3 + 3 * u] * q);
  for (int u = 0; u < np; ++u) atomicAdd(&wdw[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * q);
  if (!with_j) return;
  double dqdT = e.mfac * (e.kf * e.dlkf * e.pf - e.kr * e.dlkr * e.pr);
  if (conp) {
    double of = 0.0, orr = 0.0;
    for (int u = 0; u < nr; ++u) of += g[4 + 3 * u];
    for (int u = 0; u < np; ++u) orr += g[GEN_P + 2 + 3 * u];
    dqdT -= e.mfac * (of * e.kf * e.pf - orr * e.kr * e.pr) * invT;
    if (rx_type(inf) == 1) dqdT -= q * invT;
  }
  for (int u = 0; u < nr; ++u) atomicAdd(&dwdw[(int)g[2 + 3 * u]], -g[3 + 3 * u] * dqdT);
  for (int u = 0; u < np; ++u) atomicAdd(&dwdw[(int)g[GEN_P + 3 * u]], g[GEN_P + 1 + 3 * u] * dqdT);
  for (int side = 0; side < 2; ++side) {
    const int ns = side == 0 ? nr : np;
    const double* sl = g + (side == 0 ? 2 : GEN_P);
    const double kk = side == 0 ? e.mfac * e.kf : -e.mfac * e.kr;
    for (int s = 0; s < GEN_SLOTS; ++s) {
      double d = 0.0;
      if (s < ns && kk != 0.0) {
        d = dconc_pow(C[(int)sl[3 * s]], sl[3 * s + 2], e2t);
        for (int u = 0; u < ns; ++u)
          if (u != s) d *= conc_pow(C[(int)sl[3 * u]], sl[3 * u + 2], e2t);
        d *= kk;
      }
      Dg[(GEN_SLOTS * side + s) * IIp + i] = d;
    }
  }
}
// Jacobian columns lo..hi-1 of a general reaction from its Dg slots: column 1 + j of slot species
// j gets -nu_r dq W_k / W_j on reactant rows k and +nu_p dq W_k / W_j on product rows
__device__ __noinline__ void gen_jac_cols_big(const MechView& V, int i, uint32_t inf, const double* __restrict__ Dg,
                                              int IIp, double* jb, int c0, int lo, int hi, int LDJ) {
  const double* g = V.aux() + AUXW * (rx_aux(inf) + 1);
  const int nr = (int)g[0], np = (int)g[1];
  for (int sl = 0; sl < 2 * GEN_SLOTS; ++sl) {
    const bool prod = sl >= GEN_SLOTS;
    const int u0 = sl % GEN_SLOTS;
    if (u0 >= (prod ? np : nr)) continue;
    const int j = (int)g[(prod ? GEN_P : 2) + 3 * u0];
    const int col = 1 + j;
    if (col < lo || col >= hi) continue;
    const double dqw = Dg[sl * IIp + i] * V.rwt()[j];
    double* jc = jb + (col - c0) * LDJ + 1;
    for (int u = 0; u < nr; ++u) {
      const int k = (int)g[2 + 3 * u];
      atomicAdd(&jc[k], -g[3 + 3 * u] * dqw * V.wt()[k]);
    }
    for (int u = 0; u < np; ++u) {
      const int k = (int)g[GEN_P + 3 * u];
      atomicAdd(&jc[k], g[GEN_P + 1 + 3 * u] * dqw * V.wt()[k]);
    }
  }
}

// ------------------------------------------------------------------ right-hand side
// f(t, y) for this thread's component (thread 0 = T) and, if with_j, the Jacobian into the
// workgroup's HBM slot Jg (FP32, column-major, leading dimension NT).  Same formulation as
// oracle/ckoracle.c reactor_rhs().
template <bool PL>
__device__ __forceinline__ double rhs_big(const MechView& V, const RunCtx& R, const BigLds& L, Blk& B, double t, double yl, int tid,
                          int wid, int lane, int n, int NB, bool with_j, float* __restrict__ Jg, double* __restrict__ Dg,
                          const int* __restrict__ jptr, const uint32_t* __restrict__ jent) {
  const int KK = V.KK, KKp = V.KKp, IIp = V.IIp;
  const int sp_one = KKp - 1;
  const bool isp = tid >= 1 && tid <= KK;
  const int s = isp ? tid - 1 : 0;
  const double rw = isp ? V.rwt()[s] : 0.0;
  const double Wk = isp ? V.wt()[s] : 0.0;
  const double Yk = isp ? yl : 0.0;
  double T = yl;
  const double sumYW = bsum_bcast(B, Yk * rw, T, 0, tid, wid, lane);
  double dTdt_given = 0.0;
  if (R.ntp > 0) profile_eval(R.cfg, R.ntp, t, R.tsel, T, T, dTdt_given);  // TPRO: T(t) is given
  const double Wbar = 1.0 / sumYW;
  const int conp = R.conp;
  double rho, P, V_, dVdt = 0.0, dPdt = 0.0;
  if (R.pfr) {  // plug flow in x (ckmi_reactor.hpp pfr_pressure)
    double dPdx;
    P = pfr_pressure(R.cfg, R.npv, R.G, R.Pm, t, R.tsel, T, Wbar, dPdx);
    rho = P * Wbar / (RU * T);
    V_ = R.G / rho;
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
  const float jsx = R.pfr ? (float)(rho / R.G) : 1.0f;  // plug flow: d/dx = (rho / G) d/dt
  const double lnT = log(T), invT = 1.0 / T, lnPRT = LN_PATM_RU - lnT;
  double* C = lds_at<double>(L.C);
  double* gRT = lds_at<double>(L.gRT);
  double* hRT = lds_at<double>(L.hRT);
  double* wdw = lds_at<double>(L.wdot) + wid * KKp;
  double* dwdw = lds_at<double>(L.dwdT) + wid * KKp;
  Thermo7 th;
  th.cpR = th.hRT = th.sR = 0.0;
  if (isp) {
    th = nasa7_img(V, s, T, lnT, invT);
    C[s] = rho * Yk * rw;
    gRT[s] = th.hRT - th.sR;
    hRT[s] = th.hRT;
  } else if (tid == 0) {  // the dummy slot of the unit-coefficient reaction tables
    C[sp_one] = 1.0;
    gRT[sp_one] = 0.0;
    hRT[sp_one] = 0.0;
  }
  for (int k = lane; k < KKp; k += WAVE) {
    wdw[k] = 0.0;
    dwdw[k] = 0.0;
  }
  const double Ctot = rho * sumYW;
  __syncthreads();
  for (int g = tid; g < V.G; g += NT) {
    double m = Ctot;
    for (int p = V.gptr()[g]; p < V.gptr()[g + 1]; ++p) m += V.geff()[p] * C[V.gsp()[p]];
    lds_at<double>(L.Mg)[g] = m;
  }
  __syncthreads();
  const double* Mg = lds_at<const double>(L.Mg);
  for (int base = wid * WAVE; base < IIp; base += NT) {
    const int i = base + lane;
    const uint32_t inf = V.info()[i];
    const int nr = rx_nr(inf), np = rx_np(inf);
    if constexpr (PL) {
      if (inf & RX_GEN) {  // FORD / RORD / non-integral coefficients: real nu and orders
        gen_rhs_big(V, R, i, inf, T, lnT, invT, lnPRT, P, C, gRT, hRT, Mg, wdw, dwdw, conp, with_j, Dg, IIp);
        continue;
      }
    }
    if (nr + np == 0) continue;
    const uint32_t rs = V.rsp()[i], ps = V.psp()[i];
    const Rxn e = eval_rxn_img<PL>(V, i, inf, rs, ps, 0u, T, lnT, invT, lnPRT, P, C, gRT, hRT, Mg, with_j, R.pslot,
                                   R.plnf, R.gfac);
    const double q = e.mfac * (e.kf * e.pf - e.kr * e.pr);
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (u < nr) atomicAdd(&wdw[sp_of(rs, u)], -q);
      if (u < np) atomicAdd(&wdw[sp_of(ps, u)], q);
    }
    if (with_j) {
      double dqdT = e.mfac * (e.kf * e.dlkf * e.pf - e.kr * e.dlkr * e.pr);
      if (conp) {
        dqdT -= e.mfac * (nr * e.kf * e.pf - np * e.kr * e.pr) * invT;
        if (rx_type(inf) == 1) dqdT -= q * invT;
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if (u < nr) atomicAdd(&dwdw[sp_of(rs, u)], -dqdT);
        if (u < np) atomicAdd(&dwdw[sp_of(ps, u)], dqdT);
      }
      // dq/dC_j for every reactant slot (forward) and product slot (reverse): the product of the
      // other three slots' concentrations
      const double kf = e.mfac * e.kf, kr = -e.mfac * e.kr;
      {
        const double c0 = C[sp_of(rs, 0)], c1 = C[sp_of(rs, 1)], c2 = C[sp_of(rs, 2)], c3 = C[sp_of(rs, 3)];
        Dg[0 * IIp + i] = kf * (c1 * c2 * c3);
        Dg[1 * IIp + i] = kf * (c0 * c2 * c3);
        Dg[2 * IIp + i] = kf * (c0 * c1 * c3);
        Dg[3 * IIp + i] = kf * (c0 * c1 * c2);
      }
      {
        const double c0 = C[sp_of(ps, 0)], c1 = C[sp_of(ps, 1)], c2 = C[sp_of(ps, 2)], c3 = C[sp_of(ps, 3)];
        Dg[4 * IIp + i] = kr * (c1 * c2 * c3);
        Dg[5 * IIp + i] = kr * (c0 * c2 * c3);
        Dg[6 * IIp + i] = kr * (c0 * c1 * c3);
        Dg[7 * IIp + i] = kr * (c0 * c1 * c2);
      }
    }
  }
  __syncthreads();
  const double* wd0 = lds_at<const double>(L.wdot);
  const double wsum = isp ? ((wd0[s] + wd0[KKp + s]) + (wd0[2 * KKp + s] + wd0[3 * KKp + s])) : 0.0;
  const double rinv = 1.0 / rho;
  const double fY = wsum * Wk * rinv;
  double fl = fY;
  double cpm = 0.0, fT = 0.0, q1 = 0.0, mcp = 1.0, ck = 0.0, ekv = 0.0;
  if (R.energy == 1) {
    const double cpk = th.cpR * RU * rw;
    const double hk = th.hRT * RU * T * rw;
    ck = conp ? cpk : cpk - RU * rw;
    ekv = conp ? hk : hk - RU * T * rw;
    cpm = Yk * ck;
    double sum = ekv * fY;
    bsum2(B, cpm, sum, wid, lane);
    fT = -sum / cpm;
    if (conp) fT += dPdt / (rho * cpm);
    else fT -= P * dVdt / (V_ * rho * cpm);
    double qloss = R.qloss, area = R.areaq, dummy;
    if (R.nq > 0) profile2_eval(R.cfg, R.nq, t, R.tsel, qloss, dummy);
    if (R.na > 0) pwl_eval(R.a_t, R.a_v, R.na, t, R.tsel, area, dummy);
    mcp = R.mass * cpm;
    q1 = R.pfr ? 0.0 : R.htc * area * ERG_PER_CAL;  // plug flow: no wall heat loss on this path
    if (!R.pfr) fT -= (qloss * ERG_PER_CAL + q1 * (T - R.tamb)) / mcp;
    if (tid == 0) fl = fT;
  } else if (tid == 0) {
    fl = dTdt_given;  // 0 without TPRO
  }
  if (R.pfr && (tid != 0 || R.energy == 1 || R.ntp == 0)) fl *= rho / R.G;  // a TPRO profile is T(x)
  if (!with_j) return fl;

  // ---------------- Jacobian: column 0 (d/dT) and J[0][0]
  const double* dw0 = lds_at<const double>(L.dwdT);
  const double dws = isp ? ((dw0[s] + dw0[KKp + s]) + (dw0[2 * KKp + s] + dw0[3 * KKp + s])) : 0.0;
  const double JkT = isp ? dws * Wk * rinv + (conp ? fY * invT : 0.0) : 0.0;
  if (isp) {
    Jg[jslot(tid, 0, NB)] = (float)JkT * jsx;
    lds_at<double>(L.ek)[s] = ekv;
  }
  if (R.energy == 1) {
    const double s2 = bsum(B, ck * fY + ekv * JkT, wid, lane);  // also orders the ek writes
    if (tid == 0) Jg[0] = (float)(-s2 / cpm - q1 / mcp) * jsx;
  } else {
    if (tid == 0) Jg[0] = 0.0f;
    __syncthreads();
  }
  // ---------------- species columns 1..n-1 in blocks of jcb columns
  const int jcb = L.jcb, cpw = jcb / BW, LDJ = NT + 1;
  double* jb = lds_at<double>(L.jblk);
  const double* ek = lds_at<const double>(L.ek);
  for (int c0 = 1; c0 < n; c0 += jcb) {
    for (int idx = tid; idx < jcb * LDJ; idx += NT) jb[idx] = 0.0;
    __syncthreads();
    const int lo = c0 + wid * cpw, hi = lo + cpw;  // this wave's columns
    // the unit slots naming this wave's species lo - 1 .. hi - 2 (host-built CSR lists, ckmi.hip build_image),
    // one per lane: each wave visits only its own slots instead of all 8 IIp of them per column block (3 % on
    // configs[4]; the atomics add into each entry in another order than the all-slot walk did)
    {
      const int e0 = jptr[min(lo, n) - 1], e1 = jptr[min(hi, n) - 1];
      for (int e = e0 + lane; e < e1; e += WAVE) {
        const uint32_t en = jent[e];
        const int i = (int)(en & 0xffffu), sl = (int)(en >> 16);
        const uint32_t inf = V.info()[i];
        const int nr = rx_nr(inf), np = rx_np(inf);
        const uint32_t rs = V.rsp()[i], ps = V.psp()[i];
        const int j = sp_of(sl >= 4 ? ps : rs, sl & 3);
        const double dqw = Dg[sl * IIp + i] * V.rwt()[j];
        double* jc = jb + (1 + j - c0) * LDJ + 1;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          if (u < nr) {
            const int k = sp_of(rs, u);
            atomicAdd(&jc[k], -dqw * V.wt()[k]);
          }
          if (u < np) {
            const int k = sp_of(ps, u);
            atomicAdd(&jc[k], dqw * V.wt()[k]);
          }
        }
      }
    }
    if constexpr (PL) {  // the general reactions' slots and real coefficients (aux stream)
      for (int base = 0; base < IIp; base += WAVE) {
        const int i = base + lane;
        const uint32_t inf = V.info()[i];
        if (inf & RX_GEN) gen_jac_cols_big(V, i, inf, Dg, IIp, jb, c0, lo, hi, LDJ);
      }
    }
    __syncthreads();
    // energy row J[0][c] = -(sum_k e_k J[1+k][c]) / cpm - fT c_{c-1} / cpm  (thread c = column c)
    if (tid >= c0 && tid < c0 + jcb && tid < n) {
      double* jc = jb + (tid - c0) * LDJ;
      double r0 = 0.0;
      if (R.energy == 1) {
        double acc = 0.0;
        for (int k = 0; k < KK; ++k) acc += ek[k] * jc[1 + k];
        r0 = -acc / cpm - fT * ck / cpm;
      }
      jc[0] = r0;
    }
    __syncthreads();
    // whole float4 chunks of the J slot: item (column, chunk m, ti) = rows ti + 16 (4 m + u), u = 0..3
    // (rows >= n are the block's zeros)
    {
      const int NM = jslot_nbr(NB) / 4;
      float4* Jg4 = reinterpret_cast<float4*>(Jg);
      for (int idx = tid; idx < jcb * 16 * NM; idx += NT) {
        const int cl = idx / (16 * NM), rem = idx - cl * 16 * NM;
        const int col = c0 + cl;
        if (col >= n) continue;
        const int ti = rem & 15, m = rem >> 4, s = col & 15;
        const double* jc = jb + cl * LDJ + ti + 64 * m;
        float4 v;
        v.x = (float)jc[0] * jsx;
        v.y = (float)jc[16] * jsx;
        v.z = (float)jc[32] * jsx;
        v.w = (float)jc[48] * jsx;
        Jg4[((col >> 4) * NM + m) * NT + ((s >> 2) << 6) + ti + ((s & 3) << 4)] = v;
      }
    }
    __syncthreads();
  }
  return fl;
}

// ------------------------------------------------------------------ the kernel
template <int NB, bool PL>
__global__ __launch_bounds__(NT, 1) void big_reactor_kernel(MechImage img, BigLds L, const DevCfg* __restrict__ dcfg,
                                                           int nreact, int* __restrict__ queue,
                                                           float* __restrict__ jws, double* __restrict__ dws,
                                                           ReactorIO io) {
  const ckmi_reactor_cfg* __restrict__ cfg = &dcfg->c;
  stage_image(0, img);
  const MechView V = make_view(0, img);
  const int tid = threadIdx.x;
  const int wid = __builtin_amdgcn_readfirstlane(tid / WAVE);
  const int lane = tid % WAVE;
  const int oc = L.ctl + wid * CTL_BYTES;
  BdfS& S = *lds_at<BdfS>(oc);
  Ctl& c = *lds_at<Ctl>(oc + align16((int)sizeof(BdfS)));
  Ign& g = *lds_at<Ign>(oc + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)));
  RunCtx& R = *lds_at<RunCtx>(oc + align16((int)sizeof(BdfS)) + align16((int)sizeof(Ctl)) + align16((int)sizeof(Ign)));
  R.cfg = cfg;
  float* Jg = jws + (size_t)blockIdx.x * jslot_floats(NB);
  double* Dg = dws + (size_t)blockIdx.x * NDQ * img.IIp;
  const int KK = V.KK;
  const int n = KK + 1;
  const bool isp = tid >= 1 && tid <= KK;
  const bool act = tid < n;
  Blk B;
  B.ored = L.red;
  B.phase = 0;
  BigMat<NB, PL> M;
  BdfT<NT> b;
  b.zn.base = L.zn + tid * 8;
  BdfT<NT> b0;  // component 0 (T): its Nordsieck history, read by every thread
  b0.zn.base = L.zn;
  double fe = 0.0, y_e = 0.0, t_e = 0.0;
  bool with_j = false;
  int st = ST_NEXT;
#ifdef CKMI_PHASE_TIMERS
  unsigned long long bph[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long fph[6] = {0, 0, 0, 0, 0, 0};
  unsigned long long t_r0 = 0;
#endif

#define REQUEST_F(T_, Y_, NEXT_) \
  do {                           \
    t_e = (T_);                  \
    y_e = (Y_);                  \
    with_j = false;              \
    st = (NEXT_);                \
    want = true;                 \
  } while (0)
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
      switch (st) {
        case ST_NEXT: {
          int r = 0;
          if (tid == 0) r = atomicAdd(queue, 1);
          r = bbcast_int(B, r, 0, tid);
          if (r >= nreact) {
            st = ST_EXIT;
            break;
          }
          c.r = r;
#ifdef CKMI_PHASE_TIMERS
#pragma unroll
          for (int k = 0; k < 6; ++k) bph[k] = 0;
#pragma unroll
          for (int k = 0; k < 6; ++k) fph[k] = 0;
          t_r0 = __builtin_amdgcn_s_memtime();
#endif
          const int prob = io.problem[r];
          const double T0 = (cfg->prof_kind == 1 && cfg->energy == 2 && cfg->nprof > 0) ? cfg->prof_v[0] : io.T0[r];
          const double P0 = io.P0[r];
          double yl = 0.0;
          if (tid == 0) yl = T0;
          if (isp) yl = io.Y0[(size_t)r * KK + tid - 1];
          const double Wbar0 = 1.0 / bsum(B, isp ? yl * V.rwt()[tid - 1] : 0.0, wid, lane);
          if (dcfg->npe) {  // initial element contents: the element projection's target
            const uint64_t cnt = isp ? elem_table(V)[tid - 1] : 0ull;
            const double rw = isp ? V.rwt()[tid - 1] : 0.0;
            double v[PROJ_MMAX];
#pragma unroll
            for (int e = 0; e < PROJ_MMAX; ++e) v[e] = elem_coef(cnt, rw, e) * yl;
            bsum8(B, v, wid, lane);
#pragma unroll
            for (int e = 0; e < PROJ_MMAX; ++e) c.eb0[e] = v[e];
          }
          R.pfr = (prob == 3);
          R.conp = (prob == 1 || prob == 3);
          R.energy = cfg->energy;
          R.npv = cfg->prof_kind == 0 ? cfg->nprof : 0;
          R.ntp = (cfg->prof_kind == 1 && cfg->energy == 2) ? cfg->nprof : 0;
          R.rho0 = P0 * Wbar0 / (RU * T0);
          R.V0 = (!R.conp && R.npv > 0) ? cfg->prof_v[0] : io.V0[r];
          R.P0 = (R.conp && R.npv > 0) ? cfg->prof_v[0] : P0;
          R.mass = R.rho0 * R.V0;
          if (R.pfr) {  // plug flow: V0 is the inlet velocity u0 [cm/s]
            R.G = R.rho0 * R.V0;  // mdot / A (inlet density x u0), with or without PPRO
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
          c.avar_last = bbcast(B, yl, cfg->avar > 0 ? cfg->avar : 0, tid);
          c.T0 = T0;
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
          const double t0 = S.tn, tout = c.st_tout;
          const double tdist = fabs(tout - t0);
          const double tround = UROUND * fmax(fabs(t0), fabs(tout));
          const double hlb = 100.0 * tround;
          double hub = 0.1 * tdist;
          const double num = act ? fabs(b.zn[1]) : 0.0;
          const double den = 0.1 * fabs(b.zn[0]) + S.atol;
          const double hub_inv = bmax(B, act ? num / (den > 0 ? den : 1e-300) : 0.0, wid, lane);
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
          const double yddnrm = bwrms(B, f1, b.ewt, n, wid, lane);
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
              if (act) io.y_save[((size_t)c.r * io.nsave + c.isave) * n + tid] = b.zn[0];
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
          const double v = g.mode == 1 ? bbcast(B, fe, 0, tid) : bbcast(B, b.zn[0], g.comp, tid);
          ign_peak_update(g, 0.0, v);
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
            REQUEST_F(S.tn, b.y, ST_NLS_J);
            with_j = true;
          } else {
            S.jcur = 0;
            st = ST_SETUP;
          }
          break;
        }
        case ST_NLS_J: {
          S.nfe++;
          S.nje++;
          S.nstlj = S.nst;
          S.jcur = 1;
          st = ST_SETUP;
          break;
        }
        case ST_SETUP: {
          __syncthreads();  // the slot written by other threads' Jacobian pass
          bool ok;
          {
            BPH_T0();
            M.build(Jg, S.gamma, tid, n);
#ifdef CKMI_PHASE_TIMERS
            {  // s_memtime waits for nothing: force the loads to land before the stamp
              double chk = 0.0;
#pragma unroll
              for (int r2 = 0; r2 < NB; ++r2) chk += M.entry(r2);
              if (chk == 12345.678) bph[5] += 1;
            }
#endif
            BPH_ADD(2);
          }
          {
            BPH_T0();
#ifdef CKMI_PHASE_TIMERS
            ok = M.factor(L, B, tid, wid, lane, n, fph);
#else
            ok = M.factor(L, B, tid, wid, lane, n);
#endif
            BPH_ADD(3);
          }
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
          double x;
          {
            BPH_T0();
            x = M.solve(rhs, L, tid, wid, lane);
            BPH_ADD(4);
          }
          S.nni++;
          if (S.gamrat != 1.0) x *= 2.0 / (1.0 + S.gamrat);
          if (!act) x = 0.0;
          // the iteration's norms in one barrier (ckmi.hip reactor_kernel): del, acnrm, NNEG's negative part
          // and acnrm after NNEG's clipping
          const double z0 = b.zn[0];
          b.acor += x;
          b.y = z0 + b.acor;
          const bool neg = S.nneg && act && tid >= 1 && b.y < 0.0;
          double nv[4];
          {
            const double xe = x * b.ewt, ae = b.acor * b.ewt, ne = neg ? b.y * b.ewt : 0.0;
            const double fe2 = neg ? z0 * b.ewt : ae;
            nv[0] = xe * xe;
            nv[1] = ae * ae;
            nv[2] = ne * ne;
            nv[3] = fe2 * fe2;
          }
          bsumn<4>(B, nv, wid, lane);
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
          // One workgroup barrier per accepted step: the element sums of the corrector, the q - 1 / q + 1 norms of
          // a step that selects the next order (both from the corrector before the element projection, oracle
          // bdf_step), thread 0's h dT/dt after the history update (the TIFP monitor) as a sum, and the runaway
          // guard's maximum over the accepted state (ckmi.hip: a ballot; checked on y before the projection,
          // which moves each Y_k by a relative ~1e-10 at most)
          double ddn = 0.0, dup = 0.0;
          {
            const bool sel = S.etamax != 1.0 && S.qwait == 1;
            const bool qm = sel && S.q > 1, qp = sel && S.q != QMAX && S.saved_tq5 != 0.0;
            double cquot = 0.0;
            if (qp) {
              const double hr = S.h / S.tau[2];
              double hrL = hr;
              for (int j = 1; j < S.L; ++j) hrL *= hr;
              cquot = (S.tq[5] / S.saved_tq5) * hrL;
            }
            double znq = 0.0, lq = 0.0;
#pragma unroll
            for (int j = 0; j <= QMAX; ++j)
              if (j == S.q) {
                znq = b.zn[j];
                lq = S.l[j];
              }
            const double y = b.zn[0] + b.acor;
            const int npe = dcfg->npe;
            const uint64_t cnt = (isp && npe) ? elem_table(V)[tid - 1] : 0ull;
            const double rw = isp ? V.rwt()[tid - 1] : 0.0;
            double v[16];
#pragma unroll
            for (int e = 0; e < PROJ_MMAX; ++e) v[e] = elem_coef(cnt, rw, e) * y;
            const double a = (act && qm) ? (znq + lq * b.acor) * b.ewt : 0.0;
            const double t = (act && qp) ? (b.acor - cquot * b.zn[QMAX]) * b.ewt : 0.0;
            v[8] = a * a;
            v[9] = t * t;
            v[10] = tid == 0 ? b.zn[1] + S.l[1] * b.acor : 0.0;
#pragma unroll
            for (int e = 11; e < 16; ++e) v[e] = 0.0;
            double mx = isp ? -y : -1.0;
            if (tid == 0 && R.energy == 1 && runaway_value_bad(dcfg, y)) mx = 1e300;
            bsumn_max<16>(B, v, mx, wid, lane);
            c.rc = mx > dcfg->guard_y ? CKMI_RUN_RUNAWAY : 0;
            c.tdh = v[10];
            ddn = sqrt(v[8] / n) * S.tq[1];
            dup = sqrt(v[9] / n) * S.tq[3];
            // element conservation held to PROJ_TOL rtol (oracle elem_project), before the history update
            if (npe) {
              double r[PROJ_MMAX];
#pragma unroll
              for (int e = 0; e < PROJ_MMAX; ++e) r[e] = v[e];
              elem_project_big(V, B, npe, r, c.eb0, S.rtol, y, b.acor, tid, wid, lane, lds_at<double>(L.ek));
            }
          }
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
          if (R.pfr && R.npv == 0 && c.rc == 0) {  // plug flow past the choke point (pfr_pressure)
            double Tz = b.zn[0];
            const double sYW = bsum_bcast(B, isp ? Tz * V.rwt()[tid - 1] : 0.0, Tz, 0, tid, wid, lane);
            if (R.Pm * R.Pm - 4.0 * R.G * R.G * RU * Tz * sYW < 0.0) c.rc = CKMI_RUN_CHOKED;
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
            if (act) io.y_save[((size_t)c.r * io.nsave + c.isave) * n + tid] = ys;
            c.isave++;
          }
          // T of the accepted state (thread 0), when a monitor or the stop rule needs it; TIFP reads h dT/dt
          // from the step's fused reduction
          const bool need_T = ((g.mode == 2 || g.mode == 3) && !g.found) || (cfg->ign_stop && g.mode == 1);
          const double T_n = need_T ? bbcast(B, b.zn[0], 0, tid) : 0.0;
          if (g.mode == 1) {
            ign_peak_update(g, tn, c.tdh / S.h);
          } else if (g.mode == 4) {
            ign_peak_update(g, tn, bbcast(B, b.zn[0], g.comp, tid));
          } else if ((g.mode == 2 || g.mode == 3) && !g.found && T_n >= g.thresh) {
            // (the bbcast above ordered every thread's history update: thread 0's history is read from LDS)
            double lo = c.told, hi = tn;
            for (int it = 0; it < 60; ++it) {
              const double mid = 0.5 * (lo + hi);
              if (dky0_lane(b0, S, mid) >= g.thresh) hi = mid;
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
            if (g.mode == 1 && g.have_next && g.vlast < 0.1 * g.best && T_n > c.T0 + 200.0) {
              c.stopped = 1;
              st = ST_FINISH;
              break;
            }
          }
          bool adap = false;
          if (io.n_adap && c.nadap < io.max_adap) {
            if (cfg->asteps > 0 && c.nst % cfg->asteps == 0) adap = true;
            if (cfg->avar >= 0 && cfg->avalue > 0.0) {
              const double v = bbcast(B, b.zn[0], cfg->avar, tid);
              if (fabs(v - c.avar_last) >= cfg->avalue) adap = true;
            }
          }
          if (adap) {
            const size_t a = (size_t)c.r * io.max_adap + c.nadap;
            if (tid == 0) io.t_adap[a] = tn;
            if (act) io.y_adap[a * n + tid] = b.zn[0];
            c.nadap++;
            if (cfg->avar >= 0) c.avar_last = bbcast(B, b.zn[0], cfg->avar, tid);
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
          // final P, V (state_PV of ckmi.hip with workgroup reductions)
          double Tf = yf;
          const double sYW = bsum_bcast(B, isp ? yf * V.rwt()[tid - 1] : 0.0, Tf, 0, tid, wid, lane);
          const double Wb = 1.0 / sYW;
          double Pf, Vf, d;
          if (R.pfr) {
            Pf = pfr_pressure(R.cfg, R.npv, R.G, R.Pm, tf, tf, Tf, Wb, d);
            Vf = R.G / (Pf * Wb / (RU * Tf));
          } else if (R.conp) {
            profile_eval(R.cfg, R.npv, tf, tf, R.P0, Pf, d);
            Vf = R.rho0 * R.V0 / (Pf * Wb / (RU * Tf));
          } else {
            profile_eval(R.cfg, R.npv, tf, tf, R.V0, Vf, d);
            Pf = (R.rho0 * R.V0 / Vf) * RU * Tf / Wb;
          }
          const int r = c.r;
          while (c.isave < io.nsave) {
            if (act) io.y_save[((size_t)r * io.nsave + c.isave) * n + tid] = __builtin_nan("");
            c.isave++;
          }
          if (tid == 0) {
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
            if (io.t_stop) io.t_stop[r] = tf;
            if (io.n_adap) io.n_adap[r] = c.nadap;
          }
          if (isp) io.Y[(size_t)r * KK + tid - 1] = yf;
#ifdef CKMI_PHASE_TIMERS
          if (g_big_phase_buf && tid < 16) {  // [rhs, rhs+J, build, factor, solve, total, 6 x factor split, -]
            const unsigned long long tot = __builtin_amdgcn_s_memtime() - t_r0;
            unsigned long long v = tid == 5 ? tot : 0;
#pragma unroll
            for (int k = 0; k < 5; ++k) v = tid == k ? bph[k] : v;
#pragma unroll
            for (int k = 0; k < 6; ++k) v = tid == 6 + k ? fph[k] : v;
            g_big_phase_buf[(size_t)r * 16 + tid] = v;
          }
#endif
          st = ST_NEXT;
          break;
        }
        default:
          st = ST_EXIT;
          break;
      }
    }
    if (st == ST_EXIT) break;
    {
      BPH_T0();
      fe = rhs_big<PL>(V, R, L, B, t_e, y_e, tid, wid, lane, n, NB, with_j, Jg, Dg, img.jcol_ptr, img.jcol_ent);
#ifdef CKMI_PHASE_TIMERS
      bph[with_j ? 1 : 0] += __builtin_amdgcn_s_memtime() - _bph0;
#endif
    }
  }
#undef REQUEST_F
#undef START_BEGIN
}

// ------------------------------------------------------------------ host side
// doubles of the xpart region (solve partial sums / MFMA factorisation buffers) for an NC x NC matrix
int big_xpart_doubles(int NC) {
  const int NB = NC / 16, NBP = (NB + 1) & ~1;
  const int mfma = NB <= 11 ? std::max(2 * 4 * NC + BW * 16 * NB + BW * 4 * big_qb(NB), NB * XS) : 0;
  return std::max(NT * NBP, mfma);
}

// LDS layout for a mechanism image of img_bytes (KKp padded species, G third-body groups)
BigLds big_layout(int img_bytes, int KKp, int G, int NC, int lds_max) {
  BigLds L;
  int o = img_bytes;
  auto take = [&](int bytes) {
    const int r = o;
    o += align16(bytes);
    return r;
  };
  const int NB = NC / 16;
  L.C = take(8 * KKp);
  L.gRT = take(8 * KKp);
  L.hRT = take(8 * KKp);
  L.ek = take(8 * KKp);
  L.wdot = take(8 * BW * KKp);
  L.dwdT = take(8 * BW * KKp);
  L.Mg = take(8 * std::max(1, G));
  L.zn = take(8 * (QMAX + 1) * NT);
  const int NBP = (NB + 1) & ~1;
  const bool valu = NB > 11;  // BigMatrix (per-column steps) needs the pivot-row and column buffers
  L.prow = valu ? take(8 * BW * 4 * NBP) : 0;
  L.gcol = valu ? take(8 * 2 * 16 * NBP) : 0;
  L.phdr = take(2 * 32);  // [2] PivHdr (VALU factor) or [2] PanHdr (MFMA factor)
  L.perm = take(4 * NT);
  L.rank = take(4 * NT);
  L.bp = take(8 * 16 * NBP);
  L.red = take(8 * 2 * RED_SET);
  L.ctl = take(BW * CTL_BYTES);
  // the Jacobian column block takes what is left (multiple of BW columns, at most the matrix)
  const int LDJ = NT + 1;
  int jcb = (lds_max - align16(o) - 16) / (8 * LDJ);
  // xpart: the solve's partial sums ([NT][NBP], or [NB][XS] with the MFMA factorisation, NB <= 11); with the
  // MFMA factorisation also its panel buffers [2][4][NC], per-wave pivot rows [BW][16 NB] and per-wave
  // diagonal block rows [BW][4 QB]
  // (BigMatrixM::pan_buf / row_buf / blk_buf)
  const int xneed = 8 * big_xpart_doubles(NC);
  if (8 * LDJ * jcb < xneed && lds_max - align16(o) - 16 < xneed) jcb = 0;  // xpart must fit
  jcb = std::min(jcb, (NC + BW - 1) / BW * BW);
  jcb = jcb / BW * BW;
  L.jcb = jcb;
  L.jblk = take(std::max(8 * LDJ * std::max(jcb, 0), xneed));
  L.xpart = L.jblk;  // solves never overlap a Jacobian assembly
  L.bytes = o;
  return L;
}

template <int NB, bool PL>
int launch_big_nc(const ckmi_mech* m, int n, const DevCfg& dc, const ReactorIO& io, hipStream_t stream) {
  int lds_max = 0, ncu = 0, per_cu = 0;
  BIG_CHECK(hipDeviceGetAttribute(&lds_max, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, m->device));
  BIG_CHECK(hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, m->device));
  const BigLds L = big_layout(m->img.bytes, m->img.KKp, m->img.G, 16 * NB, lds_max);
  if (L.jcb < BW)
    return set_error(CKMI_ERR_SIZE, "mechanism image too large for the workgroup-per-reactor kernel's LDS (" +
                                        std::to_string(m->img.bytes) + " B image)");
  static thread_local std::map<std::pair<int, const void*>, int> lds_set;
  const void* fn = (const void*)big_reactor_kernel<NB, PL>;
  if (lds_set[{m->device, fn}] < L.bytes) {
    BIG_CHECK(hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, L.bytes));
    lds_set[{m->device, fn}] = L.bytes;
  }
  BIG_CHECK(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, big_reactor_kernel<NB, PL>, NT, L.bytes));
  if (per_cu < 1) return set_error(CKMI_ERR_SIZE, "workgroup-per-reactor kernel does not fit on a CU");
  const int grid = std::max(1, std::min(ncu * per_cu, n));
  const size_t jbytes = ((size_t)grid * jslot_floats(NB) * sizeof(float) + 255) & ~(size_t)255;
  const size_t dbytes = ((size_t)grid * NDQ * m->img.IIp * sizeof(double) + 255) & ~(size_t)255;
  const size_t cbytes = (sizeof(DevCfg) + 255) & ~(size_t)255;
  void* ws = nullptr;
  BIG_CHECK(hipMallocAsync(&ws, jbytes + dbytes + cbytes + 256, stream));
  char* base = (char*)ws;
  DevCfg* dcfg = (DevCfg*)(base + jbytes + dbytes);
  int* queue = (int*)(base + jbytes + dbytes + cbytes);
  auto* hc = new DevCfg(dc);
  hipError_t e = hipMemcpyAsync(dcfg, hc, sizeof(DevCfg), hipMemcpyHostToDevice, stream);
  if (e != hipSuccess) {
    delete hc;
    (void)hipFreeAsync(ws, stream);
    return set_error(CKMI_ERR_HIP, std::string("cfg copy: ") + hipGetErrorString(e));
  }
  BIG_CHECK(hipLaunchHostFunc(stream, [](void* p) { delete static_cast<DevCfg*>(p); }, hc));
  BIG_CHECK(hipMemsetAsync(queue, 0, sizeof(int), stream));
  hipLaunchKernelGGL((big_reactor_kernel<NB, PL>), dim3(grid), dim3(NT), L.bytes, stream, m->img, L, dcfg, n, queue,
                     (float*)base, (double*)(base + jbytes), io);
  BIG_CHECK(hipGetLastError());
  BIG_CHECK(hipFreeAsync(ws, stream));
  return CKMI_OK;
}

}  // namespace

int launch_big_reactors(const ckmi_mech* m, int n, const DevCfg& dc, const ReactorIO& io, hipStream_t stream) {
  const int nvar = m->KK + 1;
  if (nvar > BIG_NMAX)
    return set_error(CKMI_ERR_UNSUPPORTED, "batch reactors with more than " + std::to_string(BIG_NMAX - 1) +
                                               " species are not supported (the ROP/thermo kernels are)");
  if (m->has_plog) {
    // PLOG, chemically activated and general (FORD / RORD / fractional) reactions: the extended
    // variant, compiled for three matrix sizes (a mechanism runs in the smallest that holds it)
#ifdef CKMI_BIG_ONLY_NB
    return set_error(CKMI_ERR_UNSUPPORTED, "diagnostic build: no extended variants");
#else
    if (nvar <= 128) return launch_big_nc<8, true>(m, n, dc, io, stream);
    if (nvar <= 176) return launch_big_nc<11, true>(m, n, dc, io, stream);
    return launch_big_nc<12, true>(m, n, dc, io, stream);
#endif
  }
  switch ((nvar + 15) / 16) {  // NB: register blocks per dimension (NC = 16 NB >= n)
    case 1:
    case 2:
    case 3:
#ifdef CKMI_BIG_ONLY_NB  // diagnostics: compile one matrix size only (register-usage checks)
    default: return launch_big_nc<CKMI_BIG_ONLY_NB, false>(m, n, dc, io, stream);
#else
    case 4: return launch_big_nc<4, false>(m, n, dc, io, stream);
    case 5: return launch_big_nc<5, false>(m, n, dc, io, stream);
    case 6: return launch_big_nc<6, false>(m, n, dc, io, stream);
    case 7: return launch_big_nc<7, false>(m, n, dc, io, stream);
    case 8: return launch_big_nc<8, false>(m, n, dc, io, stream);
    case 9: return launch_big_nc<9, false>(m, n, dc, io, stream);
    case 10: return launch_big_nc<10, false>(m, n, dc, io, stream);
    case 11: return launch_big_nc<11, false>(m, n, dc, io, stream);
    default: return launch_big_nc<12, false>(m, n, dc, io, stream);
#endif
  }
}

}  // namespace ckmi

#ifdef CKMI_PHASE_TIMERS
// diagnostic build only: buf = device u64 [n][16] per-reactor phase cycles of the workgroup kernel
extern "C" int ckmi_debug_big_phase_buffer(void* buf) {
  if (hipMemcpyToSymbol(HIP_SYMBOL(ckmi::g_big_phase_buf), &buf, sizeof(buf)) != hipSuccess) return CKMI_ERR_HIP;
  return CKMI_OK;
}
#endif

// largest mechanism image (bytes, 16-B multiple) the workgroup kernel accepts for nvar = KK + 1 state variables
// (KKp padded species, G third-body groups) on a CU with lds_max bytes of LDS; -1 if none fits.  Host-only.
extern "C" int ckmi_big_max_image_bytes(int nvar, int KKp, int G, int lds_max) {
  if (nvar < 1 || nvar > ckmi::BIG_NMAX) return -1;
  const int NC = 16 * ((nvar + 15) / 16 < 4 ? 4 : (nvar + 15) / 16);
  int best = -1;
  for (int lo = 0, hi = lds_max; lo <= hi;) {
    const int mid = ((lo + hi) / 2) & ~15;
    const ckmi::BigLds L = ckmi::big_layout(mid, KKp, G, NC, lds_max);
    if (L.jcb >= ckmi::BW && L.bytes <= lds_max) {
      best = mid;
      lo = mid + 16;
    } else {
      hi = mid - 16;
    }
  }
  return best;
}
