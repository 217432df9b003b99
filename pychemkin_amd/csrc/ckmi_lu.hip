// ckmi_lu.hip -- batched dense LU factorisation with FP64 MFMA trailing updates (gfx950).
//
// The Newton iteration matrix of a batch reactor is n x n with n = KK + 1.  For GRI-3.0 (n = 54)
// the reactor kernel keeps it in one wave's VGPRs (ckmi_reactor.hpp, NewtonMatrix).  Mechanisms
// with more than 63 species (n-heptane class, n ~ 161) do not fit a
// wave; their factorisation is the right-looking blocked LU below, one workgroup of 8 waves per
// matrix, the matrix held in the workgroup's registers as 16 x 16 FP64 tiles in the
// v_mfma_f64_16x16x4_f64 C/D layout (lane l, component r: row (l >> 4) + 4 r, column l & 15):
//
//   for each 16-column panel K:
//     1. the owners of the panel tiles write them to LDS (P);
//     2. wave 0 factors the panel with partial pivoting (LAPACK dgetf2 rule: first row of
//        maximal |a|), records the swaps, reduces them to a net row permutation of at most 32
//        rows, and forms L11^-1 (unit lower, 16 x 16);
//     3. every wave applies the permutation to its tiles of the other block columns (rows
//        exchanged through LDS) and reads back its factored panel tiles;
//     4. U12 = L11^-1 A12: 4 MFMAs per tile of block row K (the tile's own C registers are the
//        B operand), written to LDS;
//     5. A22 -= L21 U12: 4 MFMAs per trailing tile, A from the panel in LDS, B from U12 in LDS.
//
// With the LDS for two panel buffers and a U12 buffer of its own (NB <= 11, LuSmem::FEW), step 5 is
// split around the next panel: every wave first updates its tiles of block column K + 1 and writes them
// straight to the other panel buffer (step 1 of panel K + 1), and waves 1..7 finish the rest of the
// update while wave 0 factors panel K + 1; four workgroup barriers per panel instead of six.
//
// The result has LAPACK dgetrf semantics (A = P L U, unit-lower L below the diagonal, U on and
// above, row interchanges applied to the whole rows) with 0-based pivot rows.  This is the
// factorisation inside the reference's closed KINAll0D_Calculate (batchreactor.py:1158) for a
// mechanism of that size; ckmi_lu_solve_batched is the matching substitution.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <string>
#include <utility>

#include "../../include/ckmi.h"

namespace {

constexpr int WAVE = 64;
constexpr int LU_WAVES = 8;  // waves per workgroup (one matrix per workgroup)
constexpr int TB = 16;       // tile edge = the 16x16x4 MFMA shape
constexpr int LU_NB_MAX = CKMI_LU_NMAX / TB;

typedef double d4 __attribute__((ext_vector_type(4)));

#ifdef CKMI_LU_PHASE  // profiling build only: wave-0 cycles per factorisation step, summed over the launch
__device__ unsigned long long g_lu_phase[12];
#define LU_PH(k)                                                              \
  do {                                                                        \
    const unsigned long long t2_ = __builtin_amdgcn_s_memtime();              \
    if (threadIdx.x == 0) ph_[k] += t2_ - t1_;                                \
    t1_ = t2_;                                                                \
  } while (0)
#define LU_PHP , unsigned long long (&ph_)[12], unsigned long long& t1_
#define LU_PHA , ph_, t1_
#else
#define LU_PH(k) (void)0
#define LU_PHP
#define LU_PHA
#endif

__device__ __forceinline__ d4 mfma16(double a, double b, d4 c) {
  return __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
}
// runtime-indexed component of a C tile, as selects (a runtime vector index would go to scratch)
__device__ __forceinline__ double comp(const d4& v, int r) { return r == 0 ? v.x : r == 1 ? v.y : r == 2 ? v.z : v.w; }
__device__ __forceinline__ void set_comp(d4& v, int r, double x) {
  v.x = r == 0 ? x : v.x;
  v.y = r == 1 ? x : v.y;
  v.z = r == 2 ? x : v.z;
  v.w = r == 3 ? x : v.w;
}
__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__device__ __forceinline__ double bcast(double v, int lane) {
  const int lo = __builtin_amdgcn_readlane(__double2loint(v), lane);
  const int hi = __builtin_amdgcn_readlane(__double2hiint(v), lane);
  return __hiloint2double(hi, lo);
}

// exact FP64 max over the wave (DPP inside rows, readlanes across them)
template <int CTRL>
__device__ __forceinline__ double dpp_mov(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), CTRL, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
__device__ __forceinline__ double wave_max(double v) {
  v = fmax(v, dpp_mov<0xB1>(v));   // quad_perm [1,0,3,2]
  v = fmax(v, dpp_mov<0x4E>(v));   // quad_perm [2,3,0,1]
  v = fmax(v, dpp_mov<0x141>(v));  // row_half_mirror
  v = fmax(v, dpp_mov<0x140>(v));  // row_mirror
  return fmax(fmax(bcast(v, 0), bcast(v, 16)), fmax(bcast(v, 32), bcast(v, 48)));
}

// row -> index of the slot tables: the 4 rows lg + 4 r (r = 0..3) of a tile lane are consecutive
__device__ __forceinline__ int slot_idx(int row) { return (row & ~15) + ((row & 3) << 2) + ((row >> 2) & 3); }

template <int NB>
struct LuSmem {
  static constexpr int NP = NB * TB;
  static constexpr int PLD = TB + 1;  // odd row stride: lanes on different rows hit different banks
  // two panel buffers (by panel parity) and a U12 buffer of its own when the LDS holds them (NB <= 11): two
  // workgroup barriers fewer per panel (the U12 step no longer overwrites the exchange buffer, and the next
  // panel's tiles go to the other buffer while slower waves still read this one)
  static constexpr bool FEW = 8 * (2 * NP * PLD + 48 * NP + TB * PLD + ((NB * NB + LU_WAVES - 1) / LU_WAVES) * 4 * WAVE) +
                                  8 * NP + 4 * TB + 4 <= 160 * 1024;
  double P[FEW ? 2 : 1][NP * PLD];    // panel block column, indexed by global row (by panel parity)
  double X[32 * NP];                  // row-exchange buffer (and the U12 block row [16][NP] without U)
  double U[FEW ? 16 * NP : 1];        // the U12 block row
  double Linv[TB * PLD];
  // per row: the slot q < 32 it is the source / destination of, or -1; stored by slot_idx so that a tile
  // lane's 4 rows (lg + 4 r, r = 0..3) are 4 consecutive ints (one 16-byte LDS read)
  alignas(16) int sslot[NP];
  alignas(16) int dslot[NP];
  int piv[TB];
  int info;
  double TS[((NB * NB + LU_WAVES - 1) / LU_WAVES) * 4 * WAVE];  // wave 0's tiles, parked during the panel
};

// L11^-1 (unit lower) by forward substitution on the identity, right-looking over columns m of
// L11: lane (i, g) holds X[i][g + 4k], k = 0..3; row m of X is lane m of each 16-lane row, brought
// to the whole row by DPP row_newbcast (the step index is a compile-time constant), so a step is
// 8 DPP moves and 4 FMAs instead of 4 LDS permutes
template <int MM>
__device__ __forceinline__ double dpp_row_bcast(double v) {
  const int lo = __builtin_amdgcn_mov_dpp(__double2loint(v), 0x150 + MM, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_mov_dpp(__double2hiint(v), 0x150 + MM, 0xf, 0xf, false);
  return __hiloint2double(hi, lo);
}
template <int... MM>
__device__ __forceinline__ void l11_steps(double (&x)[4], const double (&lm)[TB], std::integer_sequence<int, MM...>) {
  (
      [&] {
#pragma unroll
        for (int k = 0; k < 4; ++k) x[k] = fma(-lm[MM], dpp_row_bcast<MM>(x[k]), x[k]);
      }(),
      ...);
}
template <int NB>
__device__ __forceinline__ void l11_inverse(LuSmem<NB>& S, const double* Pp, int r0, int lane) {
  constexpr int PLD = LuSmem<NB>::PLD;
  const int i = lane & 15, g = lane >> 4;
  double x[4], lm[TB];
#pragma unroll
  for (int k = 0; k < 4; ++k) x[k] = (i == g + 4 * k) ? 1.0 : 0.0;
#pragma unroll
  for (int mm = 0; mm < TB - 1; ++mm) lm[mm] = i > mm ? Pp[(r0 + i) * PLD + mm] : 0.0;
  lm[TB - 1] = 0.0;
  l11_steps(x, lm, std::make_integer_sequence<int, TB - 1>{});
#pragma unroll
  for (int k = 0; k < 4; ++k) S.Linv[i * PLD + g + 4 * k] = x[k];
}


// exact int min over the wave
__device__ __forceinline__ int wave_min_i32(int v) {
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0xB1, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x4E, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x141, 0xf, 0xf, false));
  v = min(v, __builtin_amdgcn_mov_dpp(v, 0x140, 0xf, 0xf, false));
  return min(min(__builtin_amdgcn_readlane(v, 0), __builtin_amdgcn_readlane(v, 16)),
             min(__builtin_amdgcn_readlane(v, 32), __builtin_amdgcn_readlane(v, 48)));
}

// Step 2, register form (default): wave 0 holds the panel rows in VGPRs for the 16 pivot steps
// (lane l: rows r0 + l + 64 q at the start).  Rows are never moved: each carries its current
// position pos (LAPACK's row index after the interchanges so far), an interchange swaps two
// positions, and a row is finished once its position is below the current column.  So a pivot
// step is a max reduction, a position swap, the pivot row broadcast by readlane and the
// rank-1 update in registers; the rows go back to S.P at their final positions.  Wave 0 parks
// its own matrix tiles in LDS around the call (kernel register budget: 2 waves per SIMD).
// Pivots: the first position of maximal |a| (LAPACK dgetf2 / idamax).  NQ: row levels of 64 the panel
// still has (NP - 16 K rows), a template parameter so that the late panels carry 2 or 1 levels instead
// of 3 through every column step (panel_factor_lv).
template <int NB, int NQ>
__device__ __forceinline__ void panel_factor_reg(LuSmem<NB>& S, double* Pp, int K, int lane, int n LU_PHP) {
  constexpr int NP = NB * TB, PLD = LuSmem<NB>::PLD;
  constexpr int NOPOS = 1 << 30;
  const int r0 = K * TB;
  double x[NQ][TB];
  int pos[NQ];  // current position, or -1 (no row: beyond NP)
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int r = r0 + lane + WAVE * q;
    pos[q] = r < NP ? r : -1;
#pragma unroll
    for (int c = 0; c < TB; ++c) x[q][c] = r < NP ? Pp[r * PLD + c] : 0.0;
  }
  LU_PH(7);
  int zinfo = 0;  // first exactly-zero pivot column + 1 of this panel
  int pivr = 0;
#pragma unroll
  for (int c = 0; c < TB; ++c) {
    const int col = r0 + c;
    // identity padding (col >= n): the pivot is row col itself and every multiplier is 0 -- the step changes
    // nothing, so it is skipped (wave-uniform branch; n = 161: 15 of the 176 column steps)
    if (col >= n) {
      pivr = lane == c ? col : pivr;
      continue;
    }
    // this lane's best active row: largest |a|, then the smallest position; its reciprocal is
    // taken now, beside the wave reduction, instead of after the pivot row arrives
    double best = -1.0, bval = 1.0;
    int bpos = NOPOS;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const double v = pos[q] >= col ? fabs(x[q][c]) : -1.0;
      const bool take = v > best || (v == best && pos[q] < bpos);
      best = take ? v : best;
      bval = take ? x[q][c] : bval;
      bpos = take ? pos[q] : bpos;
    }
    // 1 / bval from the hardware reciprocal and two Newton steps (the IEEE division sequence is ~3x the
    // instructions; the multipliers came out bitwise the same on the A/B matrices)
    double rb = __builtin_amdgcn_rcp(bval);
    rb = fma(rb, fma(-bval, rb, 1.0), rb);
    rb = fma(rb, fma(-bval, rb, 1.0), rb);
    const double maxv = wave_max(best);
    uint64_t cand = __ballot(best == maxv);
    int p = __builtin_amdgcn_readlane(bpos, (int)__ffsll((unsigned long long)cand) - 1);
    if (__builtin_popcountll(cand) > 1) {  // ties: the first position
      p = __builtin_amdgcn_readfirstlane(wave_min_i32(best == maxv ? bpos : NOPOS));
      cand = __ballot(best == maxv && bpos == p);
    }
    p = __builtin_amdgcn_readfirstlane(p);
    pivr = lane == c ? p : pivr;  // lane c keeps the pivot of column c (one LDS store per panel)
    // the pivot row (position p) straight from its lane's registers: its level (wave-uniform after a
    // readlane) picks the register row by a scalar branch, its entries come over by readlane (no LDS
    // round trip); then it takes position col and the row at col takes p
    const int pl = (int)__ffsll((unsigned long long)cand) - 1;
    double prow[TB];
    {
      int myq = 0;
#pragma unroll
      for (int q = 1; q < NQ; ++q) myq = pos[q] == p ? q : myq;
      const int pq = __builtin_amdgcn_readlane(myq, pl);
#pragma unroll
      for (int cc = 0; cc < TB; ++cc) prow[cc] = 0.0;
#pragma unroll
      for (int q = 0; q < NQ; ++q) {
        if (pq == q) {
#pragma unroll
          for (int cc = 0; cc < TB; ++cc)
            if (cc > c) prow[cc] = bcast(x[q][cc], pl);
        }
      }
    }
#pragma unroll
    for (int q = 0; q < NQ; ++q) pos[q] = pos[q] == p ? col : (pos[q] == col ? p : pos[q]);
    // branch-free: a zero pivot column (maxv == 0, LAPACK info) multiplies by 0, rows that are not below
    // the pivot get l = 0 (x + (-0) p = x); no basic-block boundary between this column's update and the
    // next column's pivot search
    const double rp = maxv != 0.0 ? bcast(rb, pl) : 0.0;
    zinfo = (maxv == 0.0 && zinfo == 0 && col < n) ? col + 1 : zinfo;
#pragma unroll
    for (int q = 0; q < NQ; ++q) {
      const bool upd = pos[q] > col;
      const double l = upd ? x[q][c] * rp : 0.0;
      x[q][c] = upd ? l : x[q][c];
#pragma unroll
      for (int cc = 0; cc < TB; ++cc)
        if (cc > c) x[q][cc] = fma(-l, prow[cc], x[q][cc]);
    }
  }
  if (lane == 0 && zinfo != 0 && S.info == 0) S.info = zinfo;
  if (lane < TB) S.piv[lane] = pivr;
  LU_PH(8);
  // rows back to S.P at their final positions; the net permutation is read off the positions:
  // the content of row r0 + l + 64 q moved to pos[q] (at most 32 rows move), slots by prefix count
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    if (pos[q] >= 0) {
#pragma unroll
      for (int c = 0; c < TB; ++c) Pp[pos[q] * PLD + c] = x[q][c];
    }
  }
  for (int i = lane; i < NP; i += WAVE) {
    S.sslot[i] = -1;
    S.dslot[i] = -1;
  }
  int base = 0;
#pragma unroll
  for (int q = 0; q < NQ; ++q) {
    const int r = r0 + lane + WAVE * q;
    const bool moved = pos[q] >= 0 && pos[q] != r;
    const uint64_t m = __ballot(moved);
    const int sl = base + (int)__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
    if (moved) {  // (after the -1 fill: same wave, LDS order)
      S.sslot[slot_idx(r)] = sl;
      S.dslot[slot_idx(pos[q])] = sl;
    }
    base += __builtin_popcountll(m);
  }
  wave_lds_sync();
  LU_PH(10);
  l11_inverse<NB>(S, Pp, r0, lane);
  LU_PH(9);
}

// panel K with the fewest row levels that hold its NP - 16 K rows (wave-uniform choice)
template <int NB, int NQ>
__device__ __forceinline__ void panel_factor_lv(LuSmem<NB>& S, double* Pp, int K, int lane, int n LU_PHP) {
  constexpr int NP = NB * TB;
  if constexpr (NQ > 1) {
    if (NP - K * TB <= (NQ - 1) * WAVE) {
      panel_factor_lv<NB, NQ - 1>(S, Pp, K, lane, n LU_PHA);
      return;
    }
  }
  panel_factor_reg<NB, NQ>(S, Pp, K, lane, n LU_PHA);
}

template <int NB>
__global__ __launch_bounds__(LU_WAVES* WAVE) void lu_factor_kernel(int nsys, int n, double* __restrict__ A,
                                                                   int* __restrict__ ipiv, int* __restrict__ info) {
  constexpr int NP = NB * TB, PLD = LuSmem<NB>::PLD, NT = (NB * NB + LU_WAVES - 1) / LU_WAVES;
  __shared__ LuSmem<NB> S;
  const int lane = threadIdx.x & (WAVE - 1);
  const int w0 = __builtin_amdgcn_readfirstlane(threadIdx.x / WAVE);
  const int lc0 = lane & 15, lg0 = lane >> 4;

#ifdef CKMI_LU_PHASE
  unsigned long long ph_[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0}, t1_ = __builtin_amdgcn_s_memtime();
#endif
  for (int sys = blockIdx.x; sys < nsys; sys += gridDim.x) {
    double* As = A + (size_t)sys * n * n;
    d4 t[NT];
    {
      // laundered per matrix (the load offsets would otherwise be hoisted out of the sys loop)
      int w = w0, lc = lc0, lg = lg0, nl = n;
      asm volatile("" : "+s"(w), "+v"(lc), "+v"(lg), "+s"(nl));
      // tile s of wave w is tile index w + 8 s = (I, J) in row-major tile order
#pragma unroll
      for (int s = 0; s < NT; ++s) {
        const int ti = w + LU_WAVES * s;
        const int I = ti / NB, J = ti % NB;
        const int col = J * TB + lc;
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const int row = I * TB + lg + 4 * r;
          double v = row == col ? 1.0 : 0.0;  // identity padding up to a multiple of 16
          if (ti < NB * NB && row < nl && col < nl) v = As[(size_t)row * nl + col];
          t[s][r] = v;
        }
      }
    }
    if (threadIdx.x == 0) S.info = 0;
    LU_PH(0);

    for (int K = 0; K < NB; ++K) {
      // laundered per panel: keeps the per-tile indices and LDS addresses from being hoisted
      // out of the K loop and held in registers for the whole factorisation
      int w = w0, lc = lc0, lg = lg0;
      asm volatile("" : "+s"(w), "+v"(lc), "+v"(lg));
      constexpr bool FEW = LuSmem<NB>::FEW;
      constexpr bool LA = FEW;  // the trailing update split around the next panel (below)
      double* Pk = S.P[FEW ? (K & 1) : 0];
      double* Ub = FEW ? S.U : S.X;
      // 1. panel tiles (I >= K, K) to LDS (LA: written by the previous panel's update, except for K = 0)
      if (!LA || K == 0) {
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = ti / NB, J = ti % NB;
          if (ti < NB * NB && J == K && I >= K) {
#pragma unroll
            for (int r = 0; r < 4; ++r) Pk[(I * TB + lg + 4 * r) * PLD + lc] = t[s][r];
          }
        }
      }
      __syncthreads();
      LU_PH(1);
      // 2. factor the panel; LA: meanwhile waves 1..7 finish the previous panel's trailing update (the block
      // columns beyond this panel; its L21 is in the other P buffer, its U12 still in U)
      if (LA && w != 0 && K > 0) {
        const double* Pp = S.P[(K - 1) & 1];
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = ti / NB, J = ti % NB;
          if (ti < NB * NB && I > K - 1 && J > K) {
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
              t[s] = mfma16(-Pp[(I * TB + lc) * PLD + 4 * kk + lg], Ub[(4 * kk + lg) * NP + J * TB + lc], t[s]);
          }
        }
      }
      if (w == 0) {
        // park the tiles: the panel's 48 doubles per lane take their registers meanwhile
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
          for (int r = 0; r < 4; ++r) S.TS[(4 * s + r) * WAVE + lane] = t[s][r];
        panel_factor_lv<NB, (NB * TB + WAVE - 1) / WAVE>(S, Pk, K, lane, n LU_PHA);
#pragma unroll
        for (int s = 0; s < NT; ++s)
#pragma unroll
          for (int r = 0; r < 4; ++r) t[s][r] = S.TS[(4 * s + r) * WAVE + lane];
      }
      __syncthreads();
      LU_PH(2);
      // 3. row interchanges in the other block columns (sources out), factored panel back in.
      // The slot numbers of all of this wave's rows are loaded first, unconditionally (straight-line
      // LDS reads, one wait), so the lane-masked moves below do not wait on one lookup at a time.
      {
        int qs[NT][4];
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = min(ti / NB, NB - 1);
          {
            const int4 v = *reinterpret_cast<const int4*>(&S.sslot[I * TB + (lg << 2)]);  // rows lg + 4 r
            qs[s][0] = v.x;
            qs[s][1] = v.y;
            qs[s][2] = v.z;
            qs[s][3] = v.w;
          }
        }
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = ti / NB, J = ti % NB;
          if (ti < NB * NB && J != K && I >= K) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (qs[s][r] >= 0) S.X[qs[s][r] * NP + J * TB + lc] = t[s][r];
          } else if (ti < NB * NB && J == K && I >= K) {
#pragma unroll
            for (int r = 0; r < 4; ++r) t[s][r] = Pk[(I * TB + lg + 4 * r) * PLD + lc];
          }
        }
        __syncthreads();
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = min(ti / NB, NB - 1);
          {
            const int4 v = *reinterpret_cast<const int4*>(&S.dslot[I * TB + (lg << 2)]);  // rows lg + 4 r
            qs[s][0] = v.x;
            qs[s][1] = v.y;
            qs[s][2] = v.z;
            qs[s][3] = v.w;
          }
        }
#pragma unroll
        for (int s = 0; s < NT; ++s) {
          const int ti = w + LU_WAVES * s;
          const int I = ti / NB, J = ti % NB;
          if (ti < NB * NB && J != K && I >= K) {
#pragma unroll
            for (int r = 0; r < 4; ++r)
              if (qs[s][r] >= 0) t[s][r] = S.X[qs[s][r] * NP + J * TB + lc];
          }
        }
      }
      if constexpr (!FEW) __syncthreads();  // (with its own U buffer the U12 step does not overwrite X)
      LU_PH(3);
      // 4. U12 = L11^-1 A12 on block row K; U12 to LDS (Ub: U, or X reused as [16][NP])
#pragma unroll
      for (int s = 0; s < NT; ++s) {
        const int ti = w + LU_WAVES * s;
        const int I = ti / NB, J = ti % NB;
        if (ti < NB * NB && I == K && J > K) {
          d4 u = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
          for (int kk = 0; kk < 4; ++kk) u = mfma16(S.Linv[lc * PLD + 4 * kk + lg], t[s][kk], u);
          t[s] = u;
#pragma unroll
          for (int r = 0; r < 4; ++r) Ub[(lg + 4 * r) * NP + J * TB + lc] = u[r];
        }
      }
      __syncthreads();
      LU_PH(4);
      // 5. trailing update A22 -= L21 U12 (LA: waves 1..7 only the next panel's block column now, whose
      // tiles then go to the next P buffer; the rest during the next panel)
#pragma unroll
      for (int s = 0; s < NT; ++s) {
        const int ti = w + LU_WAVES * s;
        const int I = ti / NB, J = ti % NB;
        if (ti < NB * NB && I > K && J > K && (!LA || w == 0 || J == K + 1)) {
#pragma unroll
          for (int kk = 0; kk < 4; ++kk)
            t[s] = mfma16(-Pk[(I * TB + lc) * PLD + 4 * kk + lg], Ub[(4 * kk + lg) * NP + J * TB + lc], t[s]);
          if (LA && J == K + 1) {
            double* Pn = S.P[(K + 1) & 1];
#pragma unroll
            for (int r = 0; r < 4; ++r) Pn[(I * TB + lg + 4 * r) * PLD + lc] = t[s][r];
          }
        }
      }
      if (threadIdx.x < TB && K * TB + threadIdx.x < n) ipiv[(size_t)sys * n + K * TB + threadIdx.x] = S.piv[threadIdx.x];
      if constexpr (!FEW) __syncthreads();  // P, X and piv are rewritten by the next panel
      // (FEW: the next panel's tiles go to the other P buffer, and a wave reaches the next panel's X / U
      // writes only after the next panel's barriers, which every wave passes after this update)
      LU_PH(5);
    }
    // opaque copies: otherwise the 4 NT store addresses are CSE'd with the load addresses and
    // held in VGPRs through the whole factorisation
    int n_st = n, lc_st = lc0, lg = lg0, w = w0;
    double* Ast = As;
    asm volatile("" : "+s"(n_st), "+v"(lc_st), "+s"(Ast), "+v"(lg), "+s"(w));
#pragma unroll
    for (int s = 0; s < NT; ++s) {
      const int ti = w + LU_WAVES * s;
      const int I = ti / NB, J = ti % NB;
      const int col = J * TB + lc_st;
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int row = I * TB + lg + 4 * r;
        if (ti < NB * NB && row < n_st && col < n_st) Ast[(size_t)row * n_st + col] = t[s][r];
      }
    }
    if (threadIdx.x == 0) info[sys] = S.info;
    __syncthreads();  // S.info
    LU_PH(6);
  }
#ifdef CKMI_LU_PHASE
  if (threadIdx.x == 0)
    for (int k = 0; k < 12; ++k) atomicAdd(&g_lu_phase[k], ph_[k]);
#endif
}

// One wave per right-hand side: x = U^-1 L^-1 P b, in place in B[sys][n].
constexpr int SOLVE_WAVES = 4;
__global__ __launch_bounds__(SOLVE_WAVES* WAVE) void lu_solve_kernel(int nsys, int n, const double* __restrict__ LU,
                                                                     const int* __restrict__ ipiv,
                                                                     double* __restrict__ B) {
  __shared__ double xs[SOLVE_WAVES][CKMI_LU_NMAX];
  const int lane = threadIdx.x & (WAVE - 1);
  const int w = threadIdx.x / WAVE;
  const int sys = blockIdx.x * SOLVE_WAVES + w;
  if (sys >= nsys) return;  // whole wave leaves
  const double* L = LU + (size_t)sys * n * n;
  double* b = B + (size_t)sys * n;
  double* x = xs[w];
  for (int i = lane; i < n; i += WAVE) x[i] = b[i];
  wave_lds_sync();
  if (lane == 0) {
    for (int i = 0; i < n; ++i) {  // interchanges in order (dgetrs / dlaswp)
      const int p = ipiv[(size_t)sys * n + i];
      if (p != i) {
        const double tmp = x[i];
        x[i] = x[p];
        x[p] = tmp;
      }
    }
  }
  wave_lds_sync();
  for (int j = 0; j < n; ++j) {  // L y = P b (unit diagonal)
    const double yj = x[j];
    for (int i = j + 1 + lane; i < n; i += WAVE) x[i] = fma(-L[(size_t)i * n + j], yj, x[i]);
    wave_lds_sync();
  }
  for (int j = n - 1; j >= 0; --j) {  // U x = y
    const double xj = x[j] / L[(size_t)j * n + j];
    wave_lds_sync();
    if (lane == 0) x[j] = xj;
    for (int i = lane; i < j; i += WAVE) x[i] = fma(-L[(size_t)i * n + j], xj, x[i]);
    wave_lds_sync();
  }
  for (int i = lane; i < n; i += WAVE) b[i] = x[i];
}

thread_local std::string g_lu_err;

template <int NB>
hipError_t launch_factor(int nsys, int n, double* A, int* ipiv, int* info, hipStream_t st) {
  const int grid = nsys < 8192 ? nsys : 8192;
  hipLaunchKernelGGL(lu_factor_kernel<NB>, dim3(grid), dim3(LU_WAVES * WAVE), 0, st, nsys, n, A, ipiv, info);
  return hipGetLastError();
}

typedef hipError_t (*factor_fn)(int, int, double*, int*, int*, hipStream_t);
const factor_fn kFactor[LU_NB_MAX] = {launch_factor<1>, launch_factor<2>, launch_factor<3>,  launch_factor<4>,
                                      launch_factor<5>, launch_factor<6>, launch_factor<7>,  launch_factor<8>,
                                      launch_factor<9>, launch_factor<10>, launch_factor<11>, launch_factor<12>};

}  // namespace

extern "C" {

#ifdef CKMI_LU_PHASE
int ckmi_lu_phase_get(unsigned long long* out, int reset) {
  if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_lu_phase), sizeof(unsigned long long) * 12) != hipSuccess) return -1;
  if (reset) {
    unsigned long long z[12] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0};
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_lu_phase), z, sizeof(z)) != hipSuccess) return -1;
  }
  return 0;
}
#endif

const char* ckmi_lu_last_error(void) { return g_lu_err.c_str(); }

int ckmi_lu_factor_batched(int32_t nsys, int32_t n, double* A, int32_t* ipiv, int32_t* info, void* stream) {
  if (nsys < 0 || n < 1 || n > CKMI_LU_NMAX || (nsys > 0 && (!A || !ipiv || !info))) {
    g_lu_err = "ckmi_lu_factor_batched: need 1 <= n <= " + std::to_string(CKMI_LU_NMAX) + " and device pointers";
    return CKMI_ERR_ARG;
  }
  if (nsys == 0) return CKMI_OK;
  const hipError_t e = kFactor[(n + TB - 1) / TB - 1](nsys, n, A, ipiv, info, (hipStream_t)stream);
  if (e != hipSuccess) {
    g_lu_err = std::string("lu_factor_kernel launch: ") + hipGetErrorString(e);
    return CKMI_ERR_HIP;
  }
  return CKMI_OK;
}

int ckmi_lu_solve_batched(int32_t nsys, int32_t n, const double* LU, const int32_t* ipiv, double* B, void* stream) {
  if (nsys < 0 || n < 1 || n > CKMI_LU_NMAX || (nsys > 0 && (!LU || !ipiv || !B))) {
    g_lu_err = "ckmi_lu_solve_batched: need 1 <= n <= " + std::to_string(CKMI_LU_NMAX) + " and device pointers";
    return CKMI_ERR_ARG;
  }
  if (nsys == 0) return CKMI_OK;
  hipLaunchKernelGGL(lu_solve_kernel, dim3((nsys + SOLVE_WAVES - 1) / SOLVE_WAVES), dim3(SOLVE_WAVES * WAVE), 0,
                     (hipStream_t)stream, nsys, n, LU, ipiv, B);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    g_lu_err = std::string("lu_solve_kernel launch: ") + hipGetErrorString(e);
    return CKMI_ERR_HIP;
  }
  return CKMI_OK;
}

}  // extern "C"
