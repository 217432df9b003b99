// ckmi_jit.cpp -- mechanism-specialised ROP kernel, generated from the mechanism and compiled at
// run time with hipRTC for gfx950.
//
// The generic rop_kernel (ckmi.hip) puts one REACTION on each lane and walks states one at a time:
// every rate needs LDS gathers of C / g and LDS atomics into wdot, and the wave synchronises per
// state.  Here each lane owns one STATE and runs the whole mechanism as straight-line code: the
// species indices of every reaction are compile-time constants, so C_k, exp(g_k), exp(-g_k) and
// the wdot accumulators are plain registers (no LDS, no atomics, no cross-lane traffic), and the
// Arrhenius / falloff / thermo parameters are wave-uniform scalar loads from a parameter block.
// Reactions with b = E = 0 read k = A directly (no exp).  The reverse rate is kf exp(dG)
// (RT/Patm)^dnu as in the generic kernel and the oracle (an optional variant, eg = 1, uses
// products of exp(+-g_k) per species instead -- fewer exps, more registers).
//
// The source depends only on the mechanism's structure; lnA lives in the parameter block, so
// ckmi_set_afactor updates it in place without recompiling.  Compiled code objects are cached
// per process by source text.  Every reaction form of the device image is covered: elementary,
// third-body, Lindemann / Troe / SRI falloff, chemically activated, PLOG (rows in the parameter
// block, bracketing row picked per lane), Chebyshev (coefficients in the parameter block, the
// recursions unrolled), Landau-Teller (+ RLT), explicit REV, and general reactions (FORD / RORD
// orders, non-integral coefficients: C^o by the conc_pow rule of oracle/ckoracle.c, K_c from the
// real coefficients).
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <mutex>
#include <sstream>
#include <string>
#include <vector>

#include "ckmi_internal.hpp"

namespace ckmi {

namespace {

constexpr int PRM_RX = 14;  // doubles per reaction in the parameter block

std::string lit(double x) {
  char b[40];
  std::snprintf(b, sizeof(b), "%.17g", x);
  std::string s(b);
  if (s.find_first_of(".eEn") == std::string::npos) s += ".0";
  return s;
}

std::mutex g_cache_mu;
std::map<std::string, std::vector<char>> g_code_cache;  // source -> code object

const char* kPrelude = R"(
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>
#endif
__device__ __forceinline__ double jexp(double x) {
  // exp(x) = 2^k e^r, k = rint(x / ln 2), |r| <= ln2 / 2; Taylor to degree 12 (|r|^13 / 13! < 2e-16).
  // No clamp: below -745 ldexp flushes to 0, above 709 it gives inf (the int conversion saturates
  // for |x| > 1.5e9, with the same limits); NaN propagates.
  const double kd = rint(x * 1.4426950408889634);
  const double r = fma(kd, -1.9082149292705877e-10, fma(kd, -0.69314718036912382, x));
  double p = 2.08767569878680990e-09;
  p = fma(p, r, 2.50521083854417188e-08);
  p = fma(p, r, 2.75573192239858907e-07);
  p = fma(p, r, 2.75573192239858883e-06);
  p = fma(p, r, 2.48015873015873016e-05);
  p = fma(p, r, 1.98412698412698413e-04);
  p = fma(p, r, 1.38888888888888894e-03);
  p = fma(p, r, 8.33333333333333322e-03);
  p = fma(p, r, 4.16666666666666644e-02);
  p = fma(p, r, 1.66666666666666657e-01);
  p = fma(p, r, 0.5);
  p = fma(p, r, 1.0);
  p = fma(p, r, 1.0);
  return ldexp(p, (int)kd);
}
// an opaque uniform "true": each species / reaction block sits behind its own branch, so the
// instruction selector and scheduler work on one block at a time instead of the whole mechanism
__device__ __forceinline__ int jbb() {
  int f;
  asm volatile("s_mov_b32 %0, 1" : "=s"(f));
  return f;
}
// C^o for a reaction order outside {0, 1, 2, 3} (oracle/ckoracle.c conc_pow): below 1 the chord
// CFLOOR^(o-1) C under CFLOOR = 1e-14 (negative C included), otherwise C^o; above 1, 0 for C <= 0
__device__ __forceinline__ double jcpow_lt1(double c, double o, double chord) {
  return c < 1e-14 ? chord * c : jexp(o * log(c));
}
__device__ __forceinline__ double jcpow_gt1(double c, double o) { return c > 0.0 ? jexp(o * log(c)) : 0.0; }
__device__ __forceinline__ double jrcp(double x) {
  double y = __builtin_amdgcn_rcp(x);
  double e = fma(-x, y, 1.0);
  y = fma(y, e, y);
  e = fma(-x, y, 1.0);
  return fma(y, e, y);
}
)";

}  // namespace

// Generate the kernel source and the parameter block; returns false (with a reason) when the
// mechanism holds reaction types the generated kernel does not cover.
//
// Register budget: a lane holds, per species in use, C_k, exp(g_k), exp(-g_k) and the wdot
// accumulator.  Reactions are emitted sorted by their heaviest species, each species is brought in
// (Y reload, NASA-7, exp) just before its first reaction and its wdot stored right after its
// last one, so only the species of a sliding window are live (38 of 53 at most for GRI-3.0
// instead of all 53); scheduling barriers between the blocks keep the compiler from hoisting the
// whole mechanism's loads to the top.
bool jit_rop_generate(const ckmi_mech_desc* d, std::string& src, std::vector<double>& prm, std::vector<int>& lnA_off,
                      std::string& why) {
  const int KK = d->KK, II = d->II;
  if (const char* bad = ckmi::check_slots(d)) {
    why = bad;
    return false;
  }
  std::vector<int> aonly_off;
  // tuning knobs (defaults measured on MI355X, scripts/rop_jit_ab.py, profiles/r02h_jit_ab*.log):
  // reactions per basic block (8), and eg = 0: g_k in registers and one exp per reversible reaction,
  // held to 2 waves per SIMD (908 M states/s on GRI-3.0) vs eg = 1: exp(+-g_k) per species (fewer
  // instructions, more registers: 553 M at 1 wave per SIMD, 881 M at 2 with spills)
  int group = 8;
  if (const char* g = std::getenv("CKMI_JIT_GROUP")) group = std::max(1, std::atoi(g));
  int eg = 0;
  if (const char* e = std::getenv("CKMI_JIT_EG")) eg = std::atoi(e);
  int wpe = eg ? 1 : 2;  // waves per SIMD the register allocation is held to
  if (const char* w = std::getenv("CKMI_JIT_WAVES")) wpe = std::max(1, std::atoi(w));

  // general reactions: a non-integral coefficient or an order that differs from it (wide reactions
  // with integral coefficients and default orders take the unit-coefficient path below)
  std::vector<char> gen(II, 0);
  bool any_plog = false, any_cheb = false, any_lt = false, any_gen = false;
  for (int i = 0; i < II; ++i) {
    const int t = d->rtype[i];
    if (t < CKMI_RXN_ELEMENTARY || t > CKMI_RXN_LT) {
      why = "reaction type";
      return false;
    }
    if ((t == CKMI_RXN_PLOG || t == CKMI_RXN_CHEB) && (!d->plog_ptr || !d->plog_par)) {
      why = "PLOG / Chebyshev reaction without its table";
      return false;
    }
    any_plog |= t == CKMI_RXN_PLOG;
    any_cheb |= t == CKMI_RXN_CHEB;
    any_lt |= t == CKMI_RXN_LT;
    for (int u = 0; u < d->nr[i]; ++u) {
      const double nu = d->rnu[CKMI_SLOTS * i + u];
      if (nu != std::floor(nu) || nu < 1.0 || (d->ford && d->ford[CKMI_SLOTS * i + u] != nu)) gen[i] = 1;
    }
    for (int u = 0; u < d->np[i]; ++u) {
      const double nu = d->pnu[CKMI_SLOTS * i + u];
      if (nu != std::floor(nu) || nu < 1.0 || (d->rord && d->rord[CKMI_SLOTS * i + u] != nu)) gen[i] = 1;
    }
    any_gen |= gen[i] != 0;
  }
  if (any_gen) eg = 0;  // the general reactions' K_c reads g_k / RT from e_k
  const int TH = KK, RX = TH + 15 * KK;
  prm.assign(RX + PRM_RX * II, 0.0);
  lnA_off.assign(II, 0);
  for (int k = 0; k < KK; ++k) {
    prm[k] = 1.0 / d->wt[k];
    const double* t = d->thermo + 17 * k;
    prm[TH + 15 * k] = t[1];
    for (int c = 0; c < 7; ++c) {
      prm[TH + 15 * k + 1 + c] = t[3 + c];
      prm[TH + 15 * k + 8 + c] = t[10 + c];
    }
  }
  // species of each reaction (unit-coefficient expansion) and the emission order
  // rs / ps: unit-coefficient expansion (species repeated nu times); general reactions list each
  // slot species once (their coefficients and orders are read from the slots)
  std::vector<std::vector<int>> rs(II), ps(II), used(II);
  auto uses_m = [&](int i) {
    const int t = d->rtype[i];
    return t == CKMI_RXN_THIRDBODY || t == CKMI_RXN_FALLOFF || t == CKMI_RXN_CHEMACT;
  };
  for (int i = 0; i < II; ++i) {
    for (int u = 0; u < d->nr[i]; ++u) {
      const int n = gen[i] ? 1 : (int)std::lround(d->rnu[CKMI_SLOTS * i + u]);
      for (int c = 0; c < n; ++c) rs[i].push_back(d->rsp[CKMI_SLOTS * i + u]);
    }
    for (int u = 0; u < d->np[i]; ++u) {
      const int n = gen[i] ? 1 : (int)std::lround(d->pnu[CKMI_SLOTS * i + u]);
      for (int c = 0; c < n; ++c) ps[i].push_back(d->psp[CKMI_SLOTS * i + u]);
    }
    std::vector<int> u = rs[i];
    u.insert(u.end(), ps[i].begin(), ps[i].end());
    if (uses_m(i) && d->tbsp[i] >= 0) u.push_back(d->tbsp[i]);
    std::sort(u.begin(), u.end());
    u.erase(std::unique(u.begin(), u.end()), u.end());
    used[i] = u;
  }
  std::vector<int> order(II);
  for (int i = 0; i < II; ++i) order[i] = i;
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) {
    const int ma = used[a].empty() ? -1 : used[a].back(), mb = used[b].empty() ? -1 : used[b].back();
    if (ma != mb) return ma < mb;
    const int na = used[a].empty() ? -1 : used[a].front(), nb = used[b].empty() ? -1 : used[b].front();
    return na < nb;
  });
  // Opt-in (CKMI_JIT_ORDER=1, A/B only): an emission order with a narrower species window.  A species
  // is live (C_k, g_k, wdot_k in registers) from its first to its last reaction; the greedy below
  // picks next the reaction that opens the fewest species net of those it closes (fixed-seed
  // xorshift ties), best of JIT_ORDER_TRIALS runs, kept only if narrower than the sort above.  It
  // narrows GRI-3.0 from 38 to 22 live species, but measured 3.6 % SLOWER on configs[1] (887 vs 919M
  // states/s; 897M at 3 waves per SIMD, 613M at 4; profiles/r03f_ab_jit_order.log): the register
  // window is not what bounds this kernel.
  const char* oenv = std::getenv("CKMI_JIT_ORDER");
  if (oenv && oenv[0] == '1' && II > 1) {
    auto width = [&](const std::vector<int>& ord) {
      std::vector<int> f(KK, -1), l(KK, -1), ev(ord.size() + 1, 0);
      for (int pos = 0; pos < (int)ord.size(); ++pos)
        for (int k : used[ord[pos]]) {
          if (f[k] < 0) f[k] = pos;
          l[k] = pos;
        }
      for (int k = 0; k < KK; ++k)
        if (f[k] >= 0) ++ev[f[k]], --ev[l[k] + 1];
      int run = 0, w = 0;
      for (int v : ev) w = std::max(w, run += v);
      return w;
    };
    constexpr int JIT_ORDER_TRIALS = 32;
    int best_w = width(order);
    std::vector<int> cnt0(KK, 0);
    for (int i = 0; i < II; ++i)
      for (int k : used[i]) ++cnt0[k];
    for (int trial = 0; trial < JIT_ORDER_TRIALS; ++trial) {
      uint32_t rs_ = 2463534242u + 977u * (uint32_t)trial;
      auto rnd = [&]() {
        rs_ ^= rs_ << 13;
        rs_ ^= rs_ >> 17;
        rs_ ^= rs_ << 5;
        return rs_;
      };
      std::vector<int> cnt = cnt0, ord;
      std::vector<char> isopen(KK, 0), done(II, 0);
      ord.reserve(II);
      for (int step = 0; step < II; ++step) {
        int bi = -1;
        long best = 0;
        uint32_t btie = 0;
        for (int i = 0; i < II; ++i) {
          if (done[i]) continue;
          int opens = 0, closes = 0;
          for (int k : used[i]) {
            opens += !isopen[k];
            closes += cnt[k] == 1;
          }
          const long score = (long)(opens - closes) * 64 + opens;
          const uint32_t tie = rnd();
          if (bi < 0 || score < best || (score == best && tie < btie)) bi = i, best = score, btie = tie;
        }
        done[bi] = 1;
        ord.push_back(bi);
        for (int k : used[bi]) {
          isopen[k] = 1;
          if (--cnt[k] == 0) isopen[k] = 0;
        }
      }
      const int w = width(ord);
      if (w < best_w) best_w = w, order = ord;
    }
  }
  std::vector<char> needE(KK, 0), needR(KK, 0);
  for (int i = 0; i < II; ++i) {
    if (!d->rev[i] || d->has_rev[i]) continue;
    for (int k : rs[i]) needR[k] = 1;
    for (int k : ps[i]) needE[k] = 1;
  }
  std::vector<int> first(KK, -1), last(KK, -1);
  for (int pos = 0; pos < II; ++pos)
    for (int k : used[order[pos]]) {
      if (first[k] < 0) first[k] = pos;
      last[k] = pos;
    }
  // Opt-in (CKMI_JIT_WLDS=1, A/B only): the wdot accumulators in LDS instead of registers -- each
  // species gets an LDS column slot of the wave (slot * 64 + lane: every lane updates its own column,
  // conflict-free ds_add_f64, no read-modify-write wait) from its first to its last reaction, interval
  // colouring of the sliding window (38 slots, 19.5 KB per wave for GRI-3.0).  It frees registers the
  // 2-wave allocation spilled: HBM traffic per 10M-state launch 21.4 -> 17.2 GB, but 12.5 % SLOWER
  // (874 -> 764 M states/s, profiles/r04f_ab_rop_wlds.log): the scratch traffic is not what bounds it.
  std::vector<int> wslot(KK, -1);
  int nslot = 0;
  {
    std::vector<int> free_slots;
    for (int pos = 0; pos < II; ++pos) {
      for (int k : used[order[pos]])
        if (first[k] == pos) {
          if (free_slots.empty()) free_slots.push_back(nslot++);
          wslot[k] = free_slots.back();
          free_slots.pop_back();
        }
      for (int k : used[order[pos]])
        if (last[k] == pos) free_slots.push_back(wslot[k]);
    }
  }
  bool wlds = false;
  if (const char* e = std::getenv("CKMI_JIT_WLDS"))
    wlds = e[0] == '1' && nslot > 0 && (size_t)nslot * 64 * 8 * 4 * wpe <= 160 * 1024;
  std::ostringstream o;
  o << "#define CKJ_RU " << lit(1.3806504e-16 * 6.02214179e23) << "\n";  // = ckmi_device.hpp RU
  o << kPrelude;
  o << "extern \"C\" __global__ void __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(" << wpe << ", " << wpe
    << "))) ckjit_rop_k" << KK << "_i" << II << "(int n, const double* __restrict__ Tv, "
       "const double* __restrict__ Pv, const double* __restrict__ Yv, double* __restrict__ wd, "
       "double* __restrict__ cpo, double* __restrict__ ho, const double* __restrict__ prm) {\n";
  if (wlds) o << "  __shared__ double wl[" << nslot * 64 << "];\n";
  o << "  const int s0 = blockIdx.x * 64 + threadIdx.x;\n  const bool live = s0 < n;\n"
       "  const size_t s = live ? s0 : n - 1;\n  const size_t ns = n;\n";
  o << "  const double T = Tv[s], P = Pv[s];\n  const double lnT = log(T), invT = 1.0 / T;\n";
  o << "  const double rtp = CKJ_RU * T * (1.0 / 1.01325e6), prt = 1.01325e6 / (CKJ_RU * T);\n";
  if (any_plog) o << "  const double lnP = log(P);\n";
  if (any_cheb) o << "  const double lg10P = log(P) * 0.43429448190325176;\n";
  if (any_lt) o << "  const double t13 = jexp(lnT * (-1.0 / 3.0)), t23 = t13 * t13;\n";
  if (any_gen) o << "  const double lnPRT = log(prt);\n";
  o << "  double syw = 0.0, cpm = 0.0, hm = 0.0;\n";
  o << "  double";
  for (int k = 0; k < KK; ++k) o << (k ? "," : "") << " c" << k << ", e" << k << ", r" << k << ", w" << k;
  o << ";\n";
  // pass 1: mean molecular weight; third-body concentrations from the same loads
  std::map<std::vector<std::pair<int, double>>, int> gmap;
  std::vector<int> grp(II, -1);
  std::vector<char> effsp(KK, 0);
  for (int i = 0; i < II; ++i) {
    if (!uses_m(i) || d->tbsp[i] >= 0) continue;
    std::vector<std::pair<int, double>> key;
    for (int p = d->eff_ptr[i]; p < d->eff_ptr[i + 1]; ++p)
      if (d->eff_val[p] != 1.0) key.push_back({d->eff_sp[p], d->eff_val[p] - 1.0});
    std::sort(key.begin(), key.end());
    auto it = gmap.find(key);
    if (it == gmap.end()) {
      const int g = (int)gmap.size();
      gmap[key] = g;
      grp[i] = g;
    } else {
      grp[i] = it->second;
    }
    for (auto& kv : key) effsp[kv.first] = 1;
  }
  o << "  {\n";
  for (int k = 0; k < KK; ++k)
    o << "    const double y" << k << " = Yv[" << k << " * ns + s]; syw = fma(y" << k << ", prm[" << k << "], syw);\n";
  o << "    rhoc = P / (CKJ_RU * T * syw);\n";
  for (auto& kv : gmap) {
    o << "    M" << kv.second << " = rhoc * syw";
    for (auto& e : kv.first) o << " + " << lit(e.second) << " * (rhoc * y" << e.first << " * prm[" << e.first << "])";
    o << ";\n";
  }
  o << "  }\n";
  {  // declarations must precede the block above
    std::string head = o.str();
    std::string decl = "  double rhoc";
    for (auto& kv : gmap) decl += ", M" + std::to_string(kv.second);
    decl += ";\n";
    const size_t at = head.rfind("  {\n    const double y0");
    head.insert(at, decl);
    o.str("");
    o << head;
  }
  o << "  const double* Yl = Yv;\n  asm volatile(\"\" : \"+s\"(Yl));  // later Y reloads are not merged with pass 1\n";
  o << "  __builtin_amdgcn_sched_barrier(0);\n";
  // reactions per basic block: the scheduler interleaves the independent rate evaluations of a
  // group (latency hiding at one wave per SIMD); a block boundary every `group` reactions bounds
  // the live ranges.  CKMI_JIT_GROUP overrides (tuning).
  bool open = false;
  auto species = [&](int k) {
    const int b = TH + 15 * k;
    o << "  { // species " << k << "\n    const double y = Yl[" << k << " * ns + s] * prm[" << k << "];\n";
    o << "    c" << k << " = rhoc * y;\n";
    if (!wlds) o << "    w" << k << " = 0.0;\n";
    else if (wslot[k] >= 0) o << "    wl[" << wslot[k] * 64 << " + threadIdx.x] = 0.0;\n";
    o << "    const bool hi = T > prm[" << b << "];\n";
    for (int c = 0; c < 7; ++c)
      o << "    const double a" << c << " = hi ? prm[" << b + 8 + c << "] : prm[" << b + 1 + c << "];\n";
    o << "    const double cpR = fma(T, fma(T, fma(T, fma(T, a4, a3), a2), a1), a0);\n";
    o << "    const double hRT = fma(T, fma(T, fma(T, fma(T, a4 * 0.2, a3 * 0.25), a2 * (1.0 / 3.0)), a1 * 0.5), a0) + "
         "a5 * invT;\n";
    if (needE[k] || needR[k])
      o << "    const double sR = fma(a0, lnT, fma(T, fma(T, fma(T, fma(T, a4 * 0.25, a3 * (1.0 / 3.0)), a2 * 0.5), a1), "
           "a6));\n";
    if (!eg) {
      if (needE[k] || needR[k]) o << "    e" << k << " = hRT - sR;\n";  // g_k / RT
    } else if (needE[k] && needR[k]) {
      o << "    e" << k << " = jexp(hRT - sR);\n    r" << k << " = jrcp(e" << k << ");\n";
    } else if (needE[k]) {
      o << "    e" << k << " = jexp(hRT - sR);\n";
    } else if (needR[k]) {
      o << "    r" << k << " = jexp(sR - hRT);\n";
    }
    o << "    cpm = fma(y, cpR, cpm);\n    hm = fma(y, hRT, hm);\n  }\n";
  };
  auto retire = [&](int k) {
    if (!wlds) o << "  if (live) wd[" << k << " * ns + s] = w" << k << ";\n";
    else if (wslot[k] >= 0) o << "  if (live) wd[" << k << " * ns + s] = wl[" << wslot[k] * 64 << " + threadIdx.x];\n";
    else o << "  if (live) wd[" << k << " * ns + s] = 0.0;\n";
  };
  auto prod = [&](const std::vector<int>& v, const char* a) {
    std::string s;
    for (size_t j = 0; j < v.size(); ++j) s += (j ? " * " : "") + std::string(a) + std::to_string(v[j]);
    return s.empty() ? std::string("1.0") : s;
  };
  for (int pos = 0; pos < II; ++pos) {
    const int i = order[pos];
    if (pos % group == 0) {
      if (open) o << "  }\n";
      o << "  if (jbb()) {\n";
      open = true;
    }
    for (int k : used[i])
      if (first[k] == pos) species(k);
    const int o0 = RX + PRM_RX * i;
    lnA_off[i] = o0;
    const int type = d->rtype[i], ft = d->ftype[i];
    const bool fall = type == CKMI_RXN_FALLOFF || type == CKMI_RXN_CHEMACT;
    prm[o0 + 0] = d->arr[3 * i];
    prm[o0 + 1] = d->arr[3 * i + 1];
    prm[o0 + 2] = d->arr[3 * i + 2];
    prm[o0 + 3] = d->low[3 * i];
    prm[o0 + 4] = d->low[3 * i + 1];
    prm[o0 + 5] = d->low[3 * i + 2];
    for (int c = 0; c < 5; ++c) prm[o0 + 6 + c] = d->fpar[5 * i + c];
    if (fall && (ft == CKMI_FALL_TROE3 || ft == CKMI_FALL_TROE4)) {  // exp(-T / T***), exp(-T / T*): store 1/T
      prm[o0 + 7] = 1.0 / prm[o0 + 7];
      prm[o0 + 8] = 1.0 / prm[o0 + 8];
    } else if (fall && ft == CKMI_FALL_SRI) {
      prm[o0 + 8] = 1.0 / prm[o0 + 8];
    }
    prm[o0 + 11] = d->revp[3 * i];
    prm[o0 + 12] = d->revp[3 * i + 1];
    prm[o0 + 13] = d->revp[3 * i + 2];
    o << "  { // reaction " << i + 1 << "\n";
    auto P_ = [&](int off) { return "prm[" + std::to_string(off) + "]"; };
    if (type == CKMI_RXN_PLOG) {
      // rows (ln P, ln A, b, E/R) ascending in P; the bracketing pair [j, j + 1] is the count of
      // interior rows below ln P (oracle plog_rate's search), ln k linear in ln P, clamped outside
      const int r0 = d->plog_ptr[i], n = d->plog_ptr[i + 1] - r0;
      const int ab = (int)prm.size();
      for (int q = 0; q < 4 * n; ++q) prm.push_back(d->plog_par[4 * r0 + q]);
      o << "    int j = 0;\n";
      for (int q = 1; q <= n - 2; ++q) o << "    j += lnP > " << P_(ab + 4 * q) << " ? 1 : 0;\n";
      o << "    const double* t0 = prm + " << ab << " + 4 * j;\n";
      o << "    const double lk0 = t0[1] + t0[2] * lnT - t0[3] * invT;\n";
      if (n == 1) {
        o << "    const double lkinf = lk0;\n";
      } else {
        o << "    const double lk1 = t0[5] + t0[6] * lnT - t0[7] * invT;\n";
        o << "    const double w = fmin(fmax((lnP - t0[0]) / (t0[4] - t0[0]), 0.0), 1.0);\n";
        o << "    const double lkinf = lk0 + w * (lk1 - lk0);\n";
      }
      o << "    const double kfi = jexp(lkinf);\n";
    } else if (type == CKMI_RXN_CHEB) {
      // rows (NT, NP), (Tmin, Tmax, Pmin, Pmax [atm]), a[t][p]: Tr, Pr as affine maps of 1/T and
      // log10 P, both Chebyshev recursions unrolled (oracle cheb_rate)
      const double* r = d->plog_par + 4 * d->plog_ptr[i];
      const int nt = (int)r[0], npc = (int)r[1];
      const double iTmin = 1.0 / r[4], iTmax = 1.0 / r[5];
      const double lPmin = std::log10(r[6] * 1.01325e6), lPmax = std::log10(r[7] * 1.01325e6);
      const int ab = (int)prm.size();
      prm.push_back(2.0 / (iTmax - iTmin));
      prm.push_back(-(iTmin + iTmax) / (iTmax - iTmin));
      prm.push_back(2.0 / (lPmax - lPmin));
      prm.push_back(-(lPmin + lPmax) / (lPmax - lPmin));
      for (int q = 0; q < nt * npc; ++q) prm.push_back(r[8 + q]);
      o << "    const double Tr = fma(" << P_(ab) << ", invT, " << P_(ab + 1) << ");\n";
      o << "    const double Pr = fma(" << P_(ab + 2) << ", lg10P, " << P_(ab + 3) << ");\n";
      for (int q = 0; q < npc; ++q) {
        if (q == 0) o << "    const double cp0 = 1.0;\n";
        else if (q == 1) o << "    const double cp1 = Pr;\n";
        else o << "    const double cp" << q << " = 2.0 * Pr * cp" << q - 1 << " - cp" << q - 2 << ";\n";
      }
      for (int t = 0; t < nt; ++t) {
        if (t == 0) o << "    const double ct0 = 1.0;\n";
        else if (t == 1) o << "    const double ct1 = Tr;\n";
        else o << "    const double ct" << t << " = 2.0 * Tr * ct" << t - 1 << " - ct" << t - 2 << ";\n";
      }
      o << "    double lk = 0.0;\n";
      for (int t = 0; t < nt; ++t) {
        o << "    { double row = 0.0;";
        for (int q = 0; q < npc; ++q) o << " row += " << P_(ab + 4 + t * npc + q) << " * cp" << q << ";";
        o << " lk += ct" << t << " * row; }\n";
      }
      o << "    const double lkinf = lk * 2.302585092994046;\n    const double kfi = jexp(lkinf);\n";
    } else {
      std::string lk = P_(o0);
      const bool aonly = type != CKMI_RXN_LT && d->arr[3 * i + 1] == 0.0 && d->arr[3 * i + 2] == 0.0;
      if (d->arr[3 * i + 1] != 0.0) lk += " + " + P_(o0 + 1) + " * lnT";
      if (d->arr[3 * i + 2] != 0.0) lk += " - " + P_(o0 + 2) + " * invT";
      if (type == CKMI_RXN_LT) lk += " + " + P_(o0 + 3) + " * t13 + " + P_(o0 + 4) + " * t23";
      if (aonly) {  // k = A: slot 1 holds A itself (kept in step with ln A by ckmi_set_afactor)
        prm[o0 + 1] = std::exp(d->arr[3 * i]);
        aonly_off.push_back(o0);
        o << "    const double lkinf = " << lk << ";\n    const double kfi = " << P_(o0 + 1) << ";\n";
      } else {
        o << "    const double lkinf = " << lk << ";\n    const double kfi = jexp(lkinf);\n";
      }
    }
    std::string mc;
    if (uses_m(i)) mc = d->tbsp[i] >= 0 ? "c" + std::to_string(d->tbsp[i]) : "M" + std::to_string(grp[i]);
    if (fall) {
      // falloff: the slot's Arrhenius is k_inf and LOW k0, Pr = k0 [M] / k_inf, k = k_inf Pr / (1 + Pr) F;
      // chemically activated: the slot's Arrhenius is k0 and HIGH k_inf, Pr = k0 [M] / k_inf,
      // k = k0 F / (1 + Pr)
      const bool ca = type == CKMI_RXN_CHEMACT;
      o << "    const double Mc = " << mc << ";\n";
      o << "    const double lnlim = " << P_(o0 + 3) << " + " << P_(o0 + 4) << " * lnT - " << P_(o0 + 5) << " * invT;\n";
      o << "    const double lnPr = " << (ca ? "lkinf - lnlim" : "lnlim - lkinf") << " + log(Mc > 1e-300 ? Mc : 1e-300);\n";
      o << "    const double Pr = jexp(lnPr);\n    double F = 1.0;\n";
      if (ft == CKMI_FALL_TROE3 || ft == CKMI_FALL_TROE4) {
        o << "    {\n      const double lPr = fmax(lnPr * 0.43429448190325176, -300.0);\n";
        o << "      const double fa = " << P_(o0 + 6) << ";\n";
        o << "      double Fc = (1.0 - fa) * jexp(-T * " << P_(o0 + 7) << ") + fa * jexp(-T * " << P_(o0 + 8) << ");\n";
        if (ft == CKMI_FALL_TROE4) o << "      Fc += jexp(-" << P_(o0 + 9) << " * invT);\n";
        o << "      const double lnFc = log(Fc > 1e-300 ? Fc : 1e-300);\n";
        o << "      const double lFc = lnFc * 0.43429448190325176;\n";
        o << "      const double c = -0.4 - 0.67 * lFc, nn = 0.75 - 1.27 * lFc;\n";
        o << "      const double f1 = (lPr + c) / (nn - 0.14 * (lPr + c));\n";
        o << "      F = jexp(lnFc / (1.0 + f1 * f1));\n    }\n";
      } else if (ft == CKMI_FALL_SRI) {
        o << "    {\n      const double lPr = fmax(lnPr * 0.43429448190325176, -300.0);\n";
        o << "      const double X = 1.0 / (1.0 + lPr * lPr);\n";
        o << "      F = " << P_(o0 + 9) << " * pow(" << P_(o0 + 6) << " * exp(-" << P_(o0 + 7)
          << " * invT) + exp(-T * " << P_(o0 + 8) << "), X) * pow(T, " << P_(o0 + 10) << ");\n    }\n";
      }
      o << "    const double kf = " << (ca ? "kfi * (1.0 / (1.0 + Pr)) * F" : "kfi * (Pr / (1.0 + Pr)) * F") << ";\n";
    } else {
      o << "    const double kf = kfi;\n";
    }
    // concentration products: unit-coefficient products, or C^order per slot (general reactions)
    auto cpow = [&](int k, double ord) -> std::string {
      const std::string c = "c" + std::to_string(k);
      if (ord == 0.0) return "1.0";
      if (ord == 1.0) return c;
      if (ord == 2.0) return "(" + c + " * " + c + ")";
      if (ord == 3.0) return "(" + c + " * " + c + " * " + c + ")";
      if (ord < 1.0) return "jcpow_lt1(" + c + ", " + lit(ord) + ", " + lit(std::pow(1e-14, ord - 1.0)) + ")";
      return "jcpow_gt1(" + c + ", " + lit(ord) + ")";
    };
    std::string pf, pr;
    if (gen[i]) {
      for (int u = 0; u < d->nr[i]; ++u) {
        const double nu = d->rnu[CKMI_SLOTS * i + u];
        pf += (u ? " * " : "") + cpow(d->rsp[CKMI_SLOTS * i + u], d->ford ? d->ford[CKMI_SLOTS * i + u] : nu);
      }
      for (int u = 0; u < d->np[i]; ++u) {
        const double nu = d->pnu[CKMI_SLOTS * i + u];
        pr += (u ? " * " : "") + cpow(d->psp[CKMI_SLOTS * i + u], d->rord ? d->rord[CKMI_SLOTS * i + u] : nu);
      }
      if (pf.empty()) pf = "1.0";
      if (pr.empty()) pr = "1.0";
    } else {
      pf = prod(rs[i], "c");
      pr = prod(ps[i], "c");
    }
    o << "    double q = kf * (" << pf << ");\n";
    if (d->rev[i]) {
      if (d->has_rev[i]) {
        std::string rl = P_(o0 + 11) + " + " + P_(o0 + 12) + " * lnT - " + P_(o0 + 13) + " * invT";
        if (type == CKMI_RXN_LT) rl += " + " + P_(o0 + 6) + " * t13 + " + P_(o0 + 7) + " * t23";  // RLT
        o << "    double kr = jexp(" << rl << ");\n";
        if (fall) o << "    kr *= kf / kfi;\n";
      } else if (gen[i]) {
        // K_c from the real coefficients: kr = kf exp(sum nu'' g - sum nu' g - dnu ln(Patm / RT))
        std::string dg;
        double dnu = 0.0;
        for (int u = 0; u < d->np[i]; ++u) {
          const double nu = d->pnu[CKMI_SLOTS * i + u];
          dg += " + " + lit(nu) + " * e" + std::to_string(d->psp[CKMI_SLOTS * i + u]);
          dnu += nu;
        }
        for (int u = 0; u < d->nr[i]; ++u) {
          const double nu = d->rnu[CKMI_SLOTS * i + u];
          dg += " - " + lit(nu) + " * e" + std::to_string(d->rsp[CKMI_SLOTS * i + u]);
          dnu -= nu;
        }
        o << "    const double kr = kf * jexp(0.0" << dg << " - " << lit(dnu) << " * lnPRT);\n";
      } else {
        // exp(dG) as products of exp(g_p) exp(-g_r) taken in (product, reactant) pairs, so that no
        // partial product leaves the FP64 range; (RT / Patm)^dnu for the mole change
        const std::vector<int>& R = rs[i];
        const std::vector<int>& Pp = ps[i];
        std::string f;
        const size_t np = std::max(R.size(), Pp.size());
        for (size_t j = 0; j < np; ++j) {
          std::string t;
          if (j < Pp.size() && j < R.size()) t = "(e" + std::to_string(Pp[j]) + " * r" + std::to_string(R[j]) + ")";
          else if (j < Pp.size()) t = "e" + std::to_string(Pp[j]);
          else t = "r" + std::to_string(R[j]);
          f += (j ? " * " : "") + t;
        }
        const int dnu = (int)Pp.size() - (int)R.size();
        if (!eg) {  // kr = kf exp(sum_p g - sum_r g) (RT/Patm)^dnu, as the generic kernel
          std::string dg;
          for (size_t j = 0; j < Pp.size(); ++j) dg += (j ? " + e" : "e") + std::to_string(Pp[j]);
          for (size_t j = 0; j < R.size(); ++j) dg += " - e" + std::to_string(R[j]);
          f = "jexp(" + dg + ")";
        }
        for (int j = 0; j < std::abs(dnu); ++j) f += dnu > 0 ? " * rtp" : " * prt";
        o << "    const double kr = kf * (" << f << ");\n";
      }
      o << "    q -= kr * (" << pr << ");\n";
    }
    if (type == CKMI_RXN_THIRDBODY) o << "    q *= " << mc << ";\n";
    std::map<int, double> net;
    if (gen[i]) {
      for (int u = 0; u < d->nr[i]; ++u) net[d->rsp[CKMI_SLOTS * i + u]] -= d->rnu[CKMI_SLOTS * i + u];
      for (int u = 0; u < d->np[i]; ++u) net[d->psp[CKMI_SLOTS * i + u]] += d->pnu[CKMI_SLOTS * i + u];
    } else {
      for (int k : rs[i]) net[k] -= 1.0;
      for (int k : ps[i]) net[k] += 1.0;
    }
    for (auto& kv : net) {
      if (kv.second == 0.0) continue;
      if (wlds) {
        const std::string a = "&wl[" + std::to_string(wslot[kv.first] * 64) + " + threadIdx.x]";
        if (kv.second == 1.0) o << "    atomicAdd(" << a << ", q);\n";
        else if (kv.second == -1.0) o << "    atomicAdd(" << a << ", -q);\n";
        else o << "    atomicAdd(" << a << ", " << lit(kv.second) << " * q);\n";
        continue;
      }
      if (kv.second == 1.0) o << "    w" << kv.first << " += q;\n";
      else if (kv.second == -1.0) o << "    w" << kv.first << " -= q;\n";
      else o << "    w" << kv.first << " = fma(" << lit(kv.second) << ", q, w" << kv.first << ");\n";
    }
    o << "  }\n";
    for (int k : used[i])
      if (last[k] == pos) retire(k);
  }
  if (open) o << "  }\n";
  for (int k = 0; k < KK; ++k)
    if (first[k] < 0) {  // in no reaction: thermo only, zero production
      species(k);
      retire(k);
    }
  o << "  if (live) {\n    if (cpo) cpo[s] = cpm * CKJ_RU;\n    if (ho) ho[s] = hm * CKJ_RU * T;\n  }\n}\n";
  src = o.str();
  return true;
}

int jit_rop_compile(const std::string& src, std::vector<char>& code, std::string& log) {
  {
    std::lock_guard<std::mutex> lk(g_cache_mu);
    auto it = g_code_cache.find(src);
    if (it != g_code_cache.end()) {
      code = it->second;
      return 0;
    }
  }
  hiprtcProgram prog;
  if (hiprtcCreateProgram(&prog, src.c_str(), "ckjit_rop.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
    log = "hiprtcCreateProgram failed";
    return 1;
  }
  // -munsafe-fp-atomics: the LDS accumulators' atomicAdd is the native ds_add_f64 (not a CAS loop)
  const char* opts[] = {"--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=fast", "-munsafe-fp-atomics"};
  const hiprtcResult rc = hiprtcCompileProgram(prog, 5, opts);
  size_t ls = 0;
  hiprtcGetProgramLogSize(prog, &ls);
  if (ls > 1) {
    log.resize(ls);
    hiprtcGetProgramLog(prog, &log[0]);
  }
  if (rc != HIPRTC_SUCCESS) {
    hiprtcDestroyProgram(&prog);
    return 2;
  }
  size_t cs = 0;
  hiprtcGetCodeSize(prog, &cs);
  code.resize(cs);
  hiprtcGetCode(prog, code.data());
  hiprtcDestroyProgram(&prog);
  std::lock_guard<std::mutex> lk(g_cache_mu);
  g_code_cache[src] = code;
  return 0;
}

}  // namespace ckmi
