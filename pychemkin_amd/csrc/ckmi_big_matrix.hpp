// ckmi_big_matrix.hpp -- the Newton matrix of the workgroup-per-reactor kernel (ckmi_big.hip), held in the
// registers of a 4-wave workgroup: the parked Jacobian slot layout, the per-column VALU Gauss-Jordan form
// (BigMatrix, NB = 12) and the blocked Gauss-Jordan on FP64 MFMA (BigMatrixM, NB <= 11).
//
// Included once, by ckmi_big.hip, inside its anonymous namespace after the workgroup layout (BigLds, NT,
// BW, XS, big_qb), the reductions (Blk) and the phase-timer macros it uses; not a stand-alone header.
// ------------------------------------------------------------------ Newton matrix in registers
// The NC x NC matrix (NC = 16 NB; identity beyond n) is spread over the workgroup so that every
// COLUMN lives in one wave: thread (w, lane), ti = lane % 16, q = lane / 16, holds the NB x NB
// elements (ti + 16 r, 16 c + 4 w + q) in a[r][c].  Column j is therefore held by the 16 lanes
// q = j % 4 of wave (j % 16) / 4, and row i's entries of the columns of wave w by its 4 lanes
// ti = i % 16.  One Gauss-Jordan step with pivot column k = 16 b + kk then needs
//   * the pivot search over column k: one wave, a DPP max inside its 16-lane row, no barrier;
//   * the raw column k (the multipliers of every row): published by that wave through LDS -- the
//     one workgroup barrier of the step;
//   * the pivot row's entries of the columns of wave w: lanes of wave w itself (wave-local LDS).
// Look-ahead: the wave owning column k + 1 updates that column first and publishes it (with its
// pivot) before finishing the rest of step k, so the search hides behind the other waves' FMAs.
// The pivot column lives in register block column b, a compile-time index in the unrolled loop
// over b.  After factor(), a[][] holds the explicit inverse of the row-permuted matrix: with p_k
// the pivot row of step k, x_k = sum_j B[p_k][j] b[p_j].
//
// J slot layout (written by rhs_big, read by build): thread t = 64 w + ti + 16 q holds element
// (i, j) = (ti + 16 r, 16 c + 4 w + q) of the matrix as its k-th value, k = c NBR + r (NBR = NB
// rounded up to 4: the row blocks of one column block, padded); the slot stores the values in float4
// chunks [k / 4][t][k % 4], so a build loads its values with NB NBR / 4 coalesced 16-byte loads, and
// a chunk holds 4 rows of one column, so the Jacobian pass writes whole chunks (16-byte stores, 256
// contiguous bytes per 16 lanes).  (Round 5's chunks [r NB + c] mixed column blocks: each 4-byte
// store filled a quarter of a chunk, 2.2x the HBM write bytes of round 4.)
__host__ __device__ constexpr int jslot_nbr(int NB) { return (NB + 3) & ~3; }
__device__ __forceinline__ int jidx(int k, int t) { return (((k >> 2) * NT + t) << 2) + (k & 3); }
__device__ __forceinline__ int jslot(int i, int j, int NB) {
  const int s = j & 15;
  const int t = ((s >> 2) << 6) + (i & 15) + ((s & 3) << 4);
  return jidx((j >> 4) * jslot_nbr(NB) + (i >> 4), t);
}
__host__ __device__ constexpr int jslot_floats(int NB) { return NB * jslot_nbr(NB) * NT; }

template <int CTRL>
__device__ __forceinline__ uint64_t dpp_mov_u64(uint64_t v) {
  const uint32_t lo = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)v, CTRL, 0xf, 0xf, false);
  const uint32_t hi = (uint32_t)__builtin_amdgcn_mov_dpp((int)(uint32_t)(v >> 32), CTRL, 0xf, 0xf, false);
  return ((uint64_t)hi << 32) | lo;
}
// max over the 16 lanes of each DPP row, in every lane of the row
__device__ __forceinline__ uint64_t row16_max_u64(uint64_t v) {
  uint64_t o;
  o = dpp_mov_u64<DPP_QUAD_1032>(v);
  v = o > v ? o : v;
  o = dpp_mov_u64<DPP_QUAD_2301>(v);
  v = o > v ? o : v;
  o = dpp_mov_u64<DPP_ROW_HALF_MIRROR>(v);
  v = o > v ? o : v;
  o = dpp_mov_u64<DPP_ROW_MIRROR>(v);
  v = o > v ? o : v;
  return v;
}

// max of a u64 over the whole wave, in every lane: DPP inside the 16-lane rows, then the gfx950 row
// swaps (permlane16_swap pairs rows 0-1 and 2-3, permlane32_swap the two halves) -- no readlane / SGPR
// round trip, no LDS
__device__ __forceinline__ uint64_t wave_max_u64_all(uint64_t v) {
  v = row16_max_u64(v);
  {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const auto l = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    const uint64_t a = ((uint64_t)h[0] << 32) | l[0], b = ((uint64_t)h[1] << 32) | l[1];
    v = a > b ? a : b;
  }
  {
    const uint32_t lo = (uint32_t)v, hi = (uint32_t)(v >> 32);
    const auto l = __builtin_amdgcn_permlane32_swap(lo, lo, false, false);
    const auto h = __builtin_amdgcn_permlane32_swap(hi, hi, false, false);
    const uint64_t a = ((uint64_t)h[0] << 32) | l[0], b = ((uint64_t)h[1] << 32) | l[1];
    v = a > b ? a : b;
  }
  return v;
}

// pivot-step header in LDS (double-buffered by step parity)
struct PivHdr {
  double piv;
  int p, ok;
};

template <int NB>
struct BigMatrix {
  static constexpr int NC = 16 * NB;
  static constexpr int NBP = (NB + 1) & ~1;  // LDS stride of the per-lane vectors (b128 pairs)
  double a[NB][NB];
  __device__ __forceinline__ double entry(int r) const { return a[r][0]; }  // phase-timer probes

  __device__ __forceinline__ void build(const float* __restrict__ J, double gamma, int tid, int n) {
    const int t = opaque_lane(tid);
    const int lane = t & 63, w = t >> 6;
    const int ti = lane & 15, q = lane >> 4;
#pragma unroll
    for (int r = 0; r < NB; ++r) {
#pragma unroll
      for (int c = 0; c < NB; ++c) {
        const int i = ti + 16 * r, j = 16 * c + 4 * w + q;
        const double jv = (i < n && j < n) ? (double)J[jidx(c * jslot_nbr(NB) + r, t)] : 0.0;
        a[r][c] = (i == j ? 1.0 : 0.0) - gamma * jv;
      }
    }
  }

  // owner wave of step k (column k held in block column c by lanes q == k % 4): pivot search over
  // the unpivoted rows and publication of the raw column + pivot into buffer k & 1
  // (C: register block column of column k -- a constant once the caller's loop over b is unrolled)
  __device__ __forceinline__ void publish(const BigLds& L, int k, int C, uint32_t pivmask, int ti, int q) const {
    double* gcol = lds_at<double>(L.gcol) + (k & 1) * 16 * NBP;
    PivHdr* hdr = lds_at<PivHdr>(L.phdr) + (k & 1);
    const int qk = k & 3;
    uint64_t key = 0;
    double best = 0.0;
    if (q == qk) {
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        double v = a[r][0];
#pragma unroll
        for (int cc = 1; cc < NB; ++cc) v = cc == C ? a[r][cc] : v;
        gcol[ti * NBP + r] = v;
        const uint64_t kr = ((uint64_t)__float_as_uint((float)fabs(v)) << 32) | (uint32_t)(0xffffffffu - (ti + 16 * r));
        if (!((pivmask >> r) & 1u) && kr > key) {
          key = kr;
          best = v;
        }
      }
    }
    key = row16_max_u64(key);
    const uint32_t klo = __builtin_amdgcn_readlane((uint32_t)key, 16 * qk);
    const uint32_t khi = __builtin_amdgcn_readlane((uint32_t)(key >> 32), 16 * qk);
    const int p = (int)(0xffffffffu - klo);
    const int src = (p & 15) + 16 * qk;  // the lane holding the pivot
    const double piv = __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(best), src),
                                        __builtin_amdgcn_readlane(__double2loint(best), src));
    if ((ti | q) == 0) {  // lane 0 of the owner wave
      hdr->piv = piv;
      hdr->p = p;
      hdr->ok = khi != 0u;
    }
  }

  // One Gauss-Jordan step k (column k in register block column b); the owner wave of step k + 1
  // (column k + 1 in block column cn, -1 = none) updates that block column first and publishes it.
  __device__ __forceinline__ void step(const BigLds& L, int k, int b, int cn, uint32_t& pivmask, bool& ok, int t,
                                       int wid, int lane
#ifdef CKMI_PHASE_TIMERS
                                       , unsigned long long (&fph)[6]
#endif
  ) {
    const int ti = lane & 15, q = lane >> 4;
    double* prow = lds_at<double>(L.prow) + wid * 4 * NBP;  // this wave's pivot-row entries [4 q][NBP]
#ifdef CKMI_PHASE_TIMERS
    unsigned long long ft = __builtin_amdgcn_s_memtime();
#define FPH(i) do { const unsigned long long f2 = __builtin_amdgcn_s_memtime(); fph[i] += f2 - ft; ft = f2; } while (0)
#else
#define FPH(i) (void)0
#endif
    __syncthreads();  // step k's column and pivot are published
    FPH(0);
    const PivHdr h = lds_at<const PivHdr>(L.phdr)[k & 1];
    const double* gcol = lds_at<const double>(L.gcol) + (k & 1) * 16 * NBP;
    const int p = __builtin_amdgcn_readfirstlane(h.p);
    const double piv = uni(h.piv);
    if (!__builtin_amdgcn_readfirstlane(h.ok)) ok = false;
    const int tip = p & 15, rp_ = p >> 4;
    const int kk = k & 15, wk = kk >> 2, qk = kk & 3;  // owner wave / lane group of column k
    // the pivot row's entries of this wave's columns: lanes ti == tip publish them wave-locally
    if (ti == tip) {
      pivmask |= 1u << rp_;
#pragma unroll
      for (int r = 0; r < NB; ++r) {
        if (r == rp_) {  // rp_ is uniform: scalar branches select the register row
#pragma unroll
          for (int c = 0; c < NB; ++c) prow[q * NBP + c] = a[r][c];
          asm volatile("" ::: "memory");  // keep the branches apart (a merged store would index a[][] dynamically)
        }
      }
    }
    if (t == 0) {
      lds_at<int>(L.perm)[k] = p;
      lds_at<int>(L.rank)[p] = k;
    }
    const double rcp = rcp_nr(piv);
    double g[NB], pv[NB];
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      const bool isp = ti == tip && r == rp_;
      g[r] = isp ? (piv - 1.0) * rcp : gcol[ti * NBP + r] * rcp;
    }
    wave_lds_sync();
#pragma unroll
    for (int c = 0; c < NB; ++c) pv[c] = prow[q * NBP + c];
    FPH(1);
    const bool colk = wid == wk && q == qk;  // this lane holds column k (block column b)
    // rank-1 update; the pivot row is scaled by 1 / piv in the same FMA form, and column k then
    // becomes the inverse's column
    if (cn >= 0) {
#pragma unroll
      for (int r = 0; r < NB; ++r) {
#pragma unroll
        for (int c = 0; c < NB; ++c)
          if (c == cn) a[r][c] = fma(-g[r], pv[c], a[r][c]);
      }
      if (cn == b && colk) {
#pragma unroll
        for (int r = 0; r < NB; ++r) {
#pragma unroll
          for (int c = 0; c < NB; ++c)
            if (c == b) a[r][c] = (ti == tip && r == rp_) ? rcp : -g[r];
        }
      }
      if (wid == (((k + 1) & 15) >> 2)) publish(L, k + 1, cn, pivmask, ti, q);
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
#pragma unroll
      for (int c = 0; c < NB; ++c)
        if (c != cn) a[r][c] = fma(-g[r], pv[c], a[r][c]);
    }
    if (cn != b && colk) {
#pragma unroll
      for (int r = 0; r < NB; ++r) {
#pragma unroll
        for (int c = 0; c < NB; ++c)
          if (c == b) a[r][c] = (ti == tip && r == rp_) ? rcp : -g[r];
      }
    }
#ifdef CKMI_PHASE_TIMERS
    {  // the update has landed before the stamp
      double chk = 0.0;
#pragma unroll
      for (int r = 0; r < NB; ++r) chk += a[r][NB - 1];
      if (chk == 12345.678) fph[2] += 1;
    }
#endif
    FPH(2);
#undef FPH
  }

  // the steps of register block column B, then the next block column (compile-time recursion keeps
  // every register index static): steps 0..14 look ahead into B, step 15 into B + 1
  template <int Bc>
  __device__ __forceinline__ void blocks(const BigLds& L, uint32_t& pivmask, bool& ok, int t, int wid, int lane
#ifdef CKMI_PHASE_TIMERS
                                         , unsigned long long (&fph)[6]
#endif
  ) {
    if constexpr (Bc < NB) {
#pragma unroll 1
      for (int kk = 0; kk < 15; ++kk) step(L, 16 * Bc + kk, Bc, Bc, pivmask, ok, t, wid, lane
#ifdef CKMI_PHASE_TIMERS
                                           , fph
#endif
        );
      step(L, 16 * Bc + 15, Bc, Bc + 1 < NB ? Bc + 1 : -1, pivmask, ok, t, wid, lane
#ifdef CKMI_PHASE_TIMERS
           , fph
#endif
      );
      blocks<Bc + 1>(L, pivmask, ok, t, wid, lane
#ifdef CKMI_PHASE_TIMERS
                     , fph
#endif
      );
    }
  }

  // Gauss-Jordan with partial pivoting (largest |a| rounded to fp32, ties to the lowest row).
  // false if a pivot column was exactly zero (the factors are then garbage).
  __device__ __forceinline__ bool factor(const BigLds& L, Blk& B, int tid, int wid, int lane, int /*n*/
#ifdef CKMI_PHASE_TIMERS
                                         , unsigned long long (&fph)[6]
#endif
  ) {
    const int t = opaque_lane(tid);
    const int ti = lane & 15, q = lane >> 4;
    uint32_t pivmask = 0u;  // bit r: row ti + 16 r has been a pivot row
    bool ok = true;
    if (wid == 0) publish(L, 0, 0, pivmask, ti, q);
    blocks<0>(L, pivmask, ok, t, wid, lane
#ifdef CKMI_PHASE_TIMERS
              , fph
#endif
    );
    return ok;
  }

  // x = M^-1 b (thread i: component i; b must be 0 for i >= n)
  __device__ __forceinline__ double solve(double bv, const BigLds& L, int tid, int wid, int lane) const {
    const int t = opaque_lane(tid);
    const int ti = lane & 15, q = lane >> 4;
    double* bp = lds_at<double>(L.bp);      // [4 w][4 q][NBP]: position j at ((j%16)/4, j%4, j/16)
    double* xp = lds_at<double>(L.xpart);   // [4 w][4 q][16 ti][NBP] partial row sums
    const int* rank = lds_at<const int>(L.rank);
    const int* perm = lds_at<const int>(L.perm);
    if (t < NC) {
      const int j = rank[t];
      bp[(((j & 15) >> 2) * 4 + (j & 3)) * NBP + (j >> 4)] = bv;
    }
    __syncthreads();
    double pv[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) pv[c] = bp[(wid * 4 + q) * NBP + c];
    double* xo = xp + ((wid * 4 + q) * 16 + ti) * NBP;
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int c = 0; c < NB; c += 2) {
        s0 = fma(a[r][c], pv[c], s0);
        if (c + 1 < NB) s1 = fma(a[r][c + 1], pv[c + 1], s1);
      }
      xo[r] = s0 + s1;
    }
    __syncthreads();
    if (t >= NC) return 0.0;
    // component t = step t's pivot row: the 16 partial sums of row perm[t], in a fixed order
    const int i = perm[t];
    const double* xi = xp + (i & 15) * NBP + (i >> 4);
    double s[4];
#pragma unroll
    for (int w = 0; w < 4; ++w)
      s[w] = (xi[((w * 4 + 0) * 16) * NBP] + xi[((w * 4 + 1) * 16) * NBP]) +
             (xi[((w * 4 + 2) * 16) * NBP] + xi[((w * 4 + 3) * 16) * NBP]);
    return (s[0] + s[1]) + (s[2] + s[3]);
  }
};

// ------------------------------------------------------------------ blocked Gauss-Jordan on MFMA
// Same factorisation as BigMatrix (explicit inverse of the row-permuted M, partial pivoting on
// |a| rounded to fp32, ties to the lowest row, identical perm / rank / solve), reorganised in
// panels of 4 steps.  The 4 columns of a panel sit in one wave (one per lane group q), which runs
// the 4 pivot steps on them alone; GJ then gives every other column j
//     a(:, j) <- a(:, j) + P'(:, 0:4) a(P, j)        (rows P = the 4 pivot rows, values before the panel)
// with P' the processed panel columns minus the unit vectors e_p (the 4 elementary transforms
// leave every vector that is zero at the pivot rows unchanged).  That rank-4 update is one
// v_mfma_f64_16x16x4f64 per 16-row block and group of 4 register tiles: the thread layout
// (row ti + 16 r, column 16 c + 4 w + q) is exactly the MFMA C/D map of a^T (col = lane & 15 = ti,
// row = (lane >> 4) + 4 e = q + 4 e) when the 4 tiles c = 4 g + e form one accumulator, so the
// registers are updated in place.  One workgroup barrier per panel instead of one per column.
//
// The panel's 4 pivot steps are the critical path (the other three waves wait at the barrier).  In
// the MFMA layout a panel column sits in 16 lanes with 11 rows each, so a step is an 11-deep serial
// key scan, a column exchange through LDS and a pivot-row gather (round 4: ~2.2k cycles per step).
// The owner therefore transposes the 4 columns once through LDS into a row-per-lane layout (lane l:
// rows l, l + 64, l + 128 of all four columns), where a step needs no LDS at all: a 3-candidate key
// per lane, one whole-wave max (DPP + row swaps), 8 readlanes of the pivot row, and FMAs on the
// lane's own registers.  The arithmetic (pivot choice, multipliers, update) is exactly that of the
// per-column form, so the factors are bitwise the same.  Panels whose columns all lie in the
// identity padding (k0 >= n) are skipped: their steps pivot on their own row and change nothing.
typedef double v4d __attribute__((ext_vector_type(4)));

struct PanHdr {
  int p[4];
  int ok;
  int pad[3];
};

template <int NB>
struct BigMatrixM {
  static constexpr int NC = 16 * NB;
  static constexpr int NG = (NB + 3) / 4;    // accumulator groups of 4 register tiles
  static constexpr int NBP = (NB + 1) & ~1;  // LDS stride of the per-lane vectors (solve)
  v4d a[NB][NG];
  __device__ __forceinline__ double entry(int r) const { return a[r][0][0]; }  // phase-timer probes

  __device__ __forceinline__ void build(const float* __restrict__ J, double gamma, int tid, int n) {
    const int t = opaque_lane(tid);
    const int lane = t & 63, w = t >> 6;
    const int ti = lane & 15, q = lane >> 4;
    constexpr int NBR = jslot_nbr(NB), NK = NB * NBR / 4;  // float4 chunks of this thread's values (jidx)
    float jv[4 * NK];
    const float4* J4 = reinterpret_cast<const float4*>(J);
#pragma unroll
    for (int kk = 0; kk < NK; ++kk) {
      const float4 v = J4[kk * NT + t];
      jv[4 * kk] = v.x;
      jv[4 * kk + 1] = v.y;
      jv[4 * kk + 2] = v.z;
      jv[4 * kk + 3] = v.w;
    }
#pragma unroll
    for (int r = 0; r < NB; ++r) {
#pragma unroll
      for (int c = 0; c < 4 * NG; ++c) {
        const int i = ti + 16 * r, j = 16 * c + 4 * w + q;
        double v = 0.0;
        if (c < NB) {
          const double jvv = (i < n && j < n) ? (double)jv[c * NBR + r] : 0.0;
          v = (i == j ? 1.0 : 0.0) - gamma * jvv;
        }
        a[r][c >> 2][c & 3] = v;
      }
    }
  }

  static constexpr int NJ = (NC + 63) / 64;  // rows per lane in the transposed panel

  // xpart during a factorisation: panel buffers [2][4 s][NC] (alternating by panel parity), per-wave pivot
  // rows [BW][4 s][4 q][NB c], per-wave diagonal-block rows [BW][4 q][QB: 16 ti x NB c]
  static constexpr int NPB = 2;
  static constexpr int QB = big_qb(NB);
  __device__ __forceinline__ static double* pan_buf(const BigLds& L, int i) {
    return lds_at<double>(L.xpart) + i * 4 * NC;
  }
  __device__ __forceinline__ static double* row_buf(const BigLds& L, int wid) {
    return lds_at<double>(L.xpart) + NPB * 4 * NC + wid * 16 * NB;
  }
  __device__ __forceinline__ static double* blk_buf(const BigLds& L, int wid) {
    return lds_at<double>(L.xpart) + NPB * 4 * NC + BW * 16 * NB + wid * 4 * QB;
  }

  // row r of the matrix has been a pivot row: bit (r & 63) of dm[r >> 6] (wave-uniform masks)
  __device__ __forceinline__ static void mark_done(uint64_t (&dm)[NJ], int p) {
    const uint64_t bit = 1ull << (p & 63);
#pragma unroll
    for (int j = 0; j < NJ; ++j) dm[j] |= (p >> 6) == j ? bit : 0ull;  // selects, not a dynamic index
  }

  // the 4 pivot steps of the panel k0 .. k0 + 3 on its columns in the row-per-lane layout (lane l: rows
  // l, l + 64, l + 128), pivots into ps
  // JN: the row group (row >> 6) of the panel's diagonal rows, a compile-time constant (k0 .. k0 + 3 lie
  // in one 16-row block, which never straddles a multiple of 64), so the natural pivot's row needs no
  // select chain
  template <int JN>
  __device__ __forceinline__ static void pivot_steps(double (&y)[NJ][4], const uint64_t (&rid)[NJ], int k0,
                                                     uint64_t (&dm)[NJ], bool& ok, int lane, int (&ps)[4]) {
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      // the pivot row's entries of the 4 panel columns (wave-uniform, from lane pl)
      double pv[4];
      int p;
      // Natural pivot first: the diagonal row k0 + s is the pivot whenever it is still free and no
      // free row's key exceeds its key (keys are unique: the row is in the low word).  That check is
      // one readlane of the row and a ballot of 3 compares per lane; the whole-wave u64 max (6
      // dependent DPP / row-swap stages) runs only when it fails.  Same pivot, same arithmetic.
      {
        const int pn = k0 + s, pnl = pn & 63;  // wave-uniform; pn >> 6 == JN
        const uint64_t dmn = dm[JN];
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) pv[s2] = bcast(y[JN][s2], pnl);
        const uint64_t kn = ((uint64_t)__float_as_uint((float)fabs(pv[s])) << 32) | (0xffffffffu - (uint32_t)pn);
        bool above = false;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint64_t kr = ((uint64_t)__float_as_uint((float)fabs(y[j][s])) << 32) | rid[j];
          const bool cand = lane + 64 * j < NC && !((dm[j] >> lane) & 1ull);
          above = above || (cand && kr > kn);
        }
        p = pn;
        if (((dmn >> pnl) & 1ull) || __builtin_amdgcn_ballot_w64(above) != 0ull) p = -1;
        else if ((uint32_t)(kn >> 32) == 0u) ok = false;
      }
      if (p < 0) {
        uint64_t key = 0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) {
          const uint64_t kr = ((uint64_t)__float_as_uint((float)fabs(y[j][s])) << 32) | rid[j];
          const bool cand = lane + 64 * j < NC && !((dm[j] >> lane) & 1ull);
          if (cand && kr > key) key = kr;
        }
        key = wave_max_u64_all(key);
        const uint32_t klo = __builtin_amdgcn_readfirstlane((uint32_t)key);
        const uint32_t khi = __builtin_amdgcn_readfirstlane((uint32_t)(key >> 32));
        if (khi == 0u) ok = false;
        p = (int)(0xffffffffu - klo);
        const int pl = p & 63, pj = p >> 6;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) {
          double v = y[0][s2];
#pragma unroll
          for (int j = 1; j < NJ; ++j) v = pj == j ? y[j][s2] : v;
          pv[s2] = bcast(v, pl);
        }
      }
      ps[s] = p;
      const double piv = pv[s];
      const double rcp = rcp_nr(piv);
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const bool isp = lane + 64 * j == p;
        const double g = isp ? (piv - 1.0) * rcp : y[j][s] * rcp;
#pragma unroll
        for (int s2 = 0; s2 < 4; ++s2) y[j][s2] = s2 == s ? (isp ? rcp : -g) : fma(-g, pv[s2], y[j][s2]);
      }
      mark_done(dm, p);
    }
  }

  // panel of steps k0 .. k0 + 3 (k0 = 16 C + 4 wo): columns in register tile C of wave wo
  template <int C>
  __device__ __forceinline__ void panel(const BigLds& L, int wo, int par, uint64_t (&dm)[NJ], bool& ok, int t, int wid,
                                        int lane
#ifdef CKMI_PHASE_TIMERS
                                        , unsigned long long (&fph)[6]
#endif
  ) {
#ifdef CKMI_PHASE_TIMERS
    unsigned long long ft = __builtin_amdgcn_s_memtime();
#define PPH(i) do { const unsigned long long f2 = __builtin_amdgcn_s_memtime(); fph[i] += f2 - ft; ft = f2; } while (0)
#else
#define PPH(i) (void)0
#endif
    constexpr int G = C >> 2, E = C & 3;
    const int ti = lane & 15, q = lane >> 4;
    const int k0 = 16 * C + 4 * wo;
    double* Pb = pan_buf(L, par);   // [4 s][NC] P of the panel
    double* Rb = row_buf(L, wid);   // [4 s][4 q][NB c] pivot rows, per wave
    PanHdr* hdr = lds_at<PanHdr>(L.phdr) + par;
    if (wid == wo) {
      // the panel's columns into Pb ([s][NC], as published below) and back, row-per-lane
#pragma unroll
      for (int r = 0; r < NB; ++r) Pb[q * NC + ti + 16 * r] = a[r][G][E];
      wave_lds_sync();
      double y[NJ][4];
      uint64_t rid[NJ];  // low key word: 0xffffffff - row (ties go to the lowest row)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = lane + 64 * j;
        rid[j] = 0xffffffffu - (uint32_t)row;
#pragma unroll
        for (int s = 0; s < 4; ++s) y[j][s] = row < NC ? Pb[s * NC + row] : 0.0;
      }
#ifdef CKMI_PHASE_TIMERS
      {  // the transposed columns have landed before the stamp
        double chk = 0.0;
#pragma unroll
        for (int j = 0; j < NJ; ++j) chk += y[j][0];
        if (chk == 12345.678) fph[2] += 1;
      }
#endif
      PPH(2);
      int ps[4];
      pivot_steps<(16 * C) / 64>(y, rid, k0, dm, ok, lane, ps);
      // the processed panel columns P (P' = P - e_p is formed when the B operand is read)
#pragma unroll
      for (int j = 0; j < NJ; ++j) {
        const int row = lane + 64 * j;
        if (row < NC) {
#pragma unroll
          for (int s = 0; s < 4; ++s) Pb[s * NC + row] = y[j][s];
        }
      }
      if (lane < 4) {
        const int pl = lane == 0 ? ps[0] : (lane == 1 ? ps[1] : (lane == 2 ? ps[2] : ps[3]));
        lds_at<int>(L.perm)[k0 + lane] = pl;
        lds_at<int>(L.rank)[pl] = k0 + lane;
        hdr->p[lane] = pl;
      }
      if (lane == 0) hdr->ok = ok ? 1 : 0;
    }
    PPH(0);
    __syncthreads();  // the panel's P' and pivots are published
    PPH(1);
    int pr[4];
#pragma unroll
    for (int s = 0; s < 4; ++s) pr[s] = __builtin_amdgcn_readfirstlane(hdr->p[s]);
    if (!__builtin_amdgcn_readfirstlane(hdr->ok)) ok = false;
    // the 4 pivot rows' entries of this wave's columns (values before the panel), wave-locally, into
    // Rb[s][q][c] (one base address per lane, compile-time offsets).  The row's register block rp is
    // wave-uniform: the diagonal block C (natural pivots, the common case: 90-97 % of the steps of the
    // stand-in's Newton matrices at small gamma) is a static register index, any other block goes
    // through a scalar branch tree
    // (64-bit inline-asm stores from one address register: the compiler otherwise materialises an
    // address per column and parks them in AGPRs; one wave's LDS operations complete in issue order,
    // so the reads after wave_lds_sync see them)
    // All four pivot rows in the diagonal register block (the common case): every lane writes its row of
    // that block (11 full-wave stores instead of 44 with 4 lanes each and 4 branches), and the A operand
    // reads the pivot rows out of it.
    double* Bk = blk_buf(L, wid);  // [4 q][QB: 16 ti x NB c]
    // The B operands (P rows of this lane's step) are loaded here, before the gather: in the MFMA loop
    // each load had been followed by a wait for it (6 LDS round trips on the critical path).  The gather's
    // asm stores (memory clobbers) keep the compiler from sinking them.
    double Bl[NB];
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) Bl[rb] = Pb[(lane >> 4) * NC + 16 * rb + (lane & 15)];
    bool allc = true;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      mark_done(dm, pr[s]);
      allc = allc && (pr[s] >> 4) == C;
    }
    const uint32_t rbq = (uint32_t)(uintptr_t)(Rb + q * NB);
    if (allc) {
      // (16 lanes of one store group: ti stride NB doubles, NB odd -> conflict-free)
      const uint32_t bkq = (uint32_t)(uintptr_t)(Bk + q * QB + ti * NB);
#pragma unroll
      for (int c = 0; c < NB; ++c)
        asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(bkq), "v"(a[C][c >> 2][c & 3]), "i"(8 * c) : "memory");
    } else {
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int tip = pr[s] & 15, rp = pr[s] >> 4;
        if (rp == C) {
          if (ti == tip) {
#pragma unroll
            for (int c = 0; c < NB; ++c)
              asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(rbq), "v"(a[C][c >> 2][c & 3]),
                           "i"(8 * (s * 4 * NB + c)) : "memory");
          }
        } else {
#pragma unroll
          for (int r = 0; r < NB; ++r) {
            if (r != C && r == rp) {  // uniform: one scalar branch selects the register row
              if (ti == tip) {
#pragma unroll
                for (int c = 0; c < NB; ++c)
                  asm volatile("ds_write_b64 %0, %1 offset:%2" : : "v"(rbq), "v"(a[r][c >> 2][c & 3]),
                               "i"(8 * (s * 4 * NB + c)) : "memory");
              }
              asm volatile("" ::: "memory");
            }
          }
        }
      }
    }
    wave_lds_sync();
    PPH(3);
    // A = U^T (lane: column j = lane & 15 of the group, panel step lane >> 4), B = P'^T
    const int sl = lane >> 4;
    const int pl = sl == 0 ? pr[0] : (sl == 1 ? pr[1] : (sl == 2 ? pr[2] : pr[3]));  // pivot row of step sl
    double A[NG];
    {
      const int j = lane & 15;
      const double* ra = allc ? Bk + (j & 3) * QB + (pl & 15) * NB + (j >> 2)
                              : Rb + ((lane >> 4) * 4 + (j & 3)) * NB + (j >> 2);
#pragma unroll
      for (int g = 0; g < NG; ++g) A[g] = 4 * g + (j >> 2) < NB ? ra[4 * g] : 0.0;
    }
    // row-block-major issue order (a group-first order that would let the next panel's owner start
    // earlier measured 1.3 % slower: DESIGN.md §5)
#pragma unroll
    for (int rb = 0; rb < NB; ++rb) {
      const int i = 16 * rb + (lane & 15);
      const double Bv = Bl[rb] - (i == pl ? 1.0 : 0.0);
#pragma unroll
      for (int g = 0; g < NG; ++g) a[rb][g] = __builtin_amdgcn_mfma_f64_16x16x4f64(A[g], Bv, a[rb][g], 0, 0, 0);
    }
#ifdef CKMI_PHASE_TIMERS
    {  // the MFMA results have landed before the stamp
      double chk = 0.0;
#pragma unroll
      for (int r = 0; r < NB; ++r) chk += a[r][NG - 1][0];
      if (chk == 12345.678) fph[4] += 1;
    }
#endif
    PPH(4);
    if (wid == wo) {  // the panel columns keep their processed values
#pragma unroll
      for (int r = 0; r < NB; ++r) a[r][G][E] = Pb[q * NC + ti + 16 * r];
    }
#ifdef CKMI_PHASE_TIMERS
    {  // the updates have landed before the stamp
      double chk = 0.0;
#pragma unroll
      for (int r = 0; r < NB; ++r) chk += a[r][0][0];
      if (chk == 12345.678) fph[2] += 1;
    }
#endif
    PPH(5);
#undef PPH
  }

#ifdef CKMI_PHASE_TIMERS
#define FPH_ARG , fph
#define FPH_PARAM , unsigned long long (&fph)[6]
#else
#define FPH_ARG
#define FPH_PARAM
#endif
  template <int C>
  __device__ __forceinline__ void panels(const BigLds& L, int n, uint64_t (&dm)[NJ], bool& ok, int t, int wid,
                                         int lane FPH_PARAM) {
    if constexpr (C < NB) {
#pragma unroll 1  // (fully unrolled: 4x the code, and the ROCm 7.2 backend crashes in AMDGPU Rewrite AGPR-Copy-MFMA)
      for (int wo = 0; wo < 4; ++wo)
        if (16 * C + 4 * wo < n) panel<C>(L, wo, (C * 4 + wo) & 1, dm, ok, t, wid, lane FPH_ARG);
      panels<C + 1>(L, n, dm, ok, t, wid, lane FPH_ARG);
    }
  }

  __device__ __forceinline__ bool factor(const BigLds& L, Blk& B, int tid, int wid, int lane, int n
#ifdef CKMI_PHASE_TIMERS
                                         , unsigned long long (&fph)[6]
#endif
  ) {
    (void)B;
    const int t = opaque_lane(tid);
    // steps of the skipped identity-padding panels pivot on their own row (published before the
    // first panel's barrier; the solve reads perm / rank after the last one)
    const int kpad = (n + 3) & ~3;
    if (t >= kpad && t < NC) {
      lds_at<int>(L.perm)[t] = t;
      lds_at<int>(L.rank)[t] = t;
    }
    uint64_t dm[NJ];
#pragma unroll
    for (int j = 0; j < NJ; ++j) dm[j] = 0ull;
    bool ok = true;
    panels<0>(L, n, dm, ok, t, wid, lane FPH_ARG);
    return ok;
  }

  // x = M^-1 b (thread i: component i; b must be 0 for i >= n) -- as BigMatrix::solve
  __device__ __forceinline__ double solve(double bv, const BigLds& L, int tid, int wid, int lane) const {
    const int t = opaque_lane(tid);
    const int ti = lane & 15, q = lane >> 4;
    double* bp = lds_at<double>(L.bp);
    double* xp = lds_at<double>(L.xpart);
    const int* rank = lds_at<const int>(L.rank);
    const int* perm = lds_at<const int>(L.perm);
    // natural order (position j at bp[j]) and partial sums [r][XS] by thread: the stores of the common
    // (natural-pivot) case and the row-sum reads are bank-conflict-free; same sums, same order as
    // BigMatrix::solve
    if (t < NC) bp[rank[t]] = bv;
    __syncthreads();
    double pv[NB];
#pragma unroll
    for (int c = 0; c < NB; ++c) pv[c] = bp[16 * c + 4 * wid + q];
    double* xo = xp + t;
#pragma unroll
    for (int r = 0; r < NB; ++r) {
      double s0 = 0.0, s1 = 0.0;
#pragma unroll
      for (int c = 0; c < NB; c += 2) {
        s0 = fma(a[r][c >> 2][c & 3], pv[c], s0);
        if (c + 1 < NB) s1 = fma(a[r][(c + 1) >> 2][(c + 1) & 3], pv[c + 1], s1);
      }
      xo[r * XS] = s0 + s1;
    }
    __syncthreads();
    if (t >= NC) return 0.0;
    const int i = perm[t];
    const double* xi = xp + (i >> 4) * XS + (i & 15);
    double s[4];
#pragma unroll
    for (int w = 0; w < 4; ++w)
      s[w] = (xi[w * 64 + 0] + xi[w * 64 + 16]) + (xi[w * 64 + 32] + xi[w * 64 + 48]);
    return (s[0] + s[1]) + (s[2] + s[3]);
  }
};

// NB = 12 (177..192 variables) keeps the per-column VALU factorisation: its MFMA form overflows
// the register file (and crashes the ROCm 7.2 backend with the VGPR-form MFMA option)
template <int NB, bool PL>
using BigMat = std::conditional_t<(NB <= 11), BigMatrixM<NB>, BigMatrix<NB>>;
