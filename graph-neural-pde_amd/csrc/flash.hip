// flash.hip — the per-edge scaled_dot attention RHS under source-grouped
// softmax (attention_norm_idx 0, upstream GRAND's default transformer RHS) as
// ONE aggregation pass over the CSR plan: the softmax group of an edge is its
// source, i.e. the row the aggregation sums into, so each row slot scores the
// edges it is about to gather, forms the group statistics itself and then runs
// K1's gather loop with the finished weights.  No [nnz] weight array, no
// separate softmax launch over the edges.  Reference:
//   SpGraphTransAttentionLayer.forward  src/function_transformer_attention.py:218-266
//     (q = Q x, k = K x, prods = q_src . k_dst / sqrt(dk) — upstream GRAND's per-edge score)
//   utils.softmax (groups = edge_index[0])  src/utils.py:116-127
//   multiply_attention (head mean, A x)     src/function_transformer_attention.py:33-41
//   ODEFuncTransformerAtt.forward            :44-59 (f = a (A x - x) [+ b x0])
//
// Per row r with edges e -> c_e, head h (scores in log2 units, s * log2(e)):
//   s_e,h = q_r,h . k_c,h / sqrt(dk)
//   M_h = max_e s_e,h,  L_h = sum_e exp(s_e,h - M_h)
//   w_e = (1/H) sum_h exp(s_e,h - M_h) / (L_h + 1e-16)        (utils.softmax + head mean)
//   ax_r = sum_e w_e x_c
//
// Work item = K1's plan item (a row of at most `chunk` edges, or a chunk of a
// hub row), RPW rows per wavefront, SL = 64/RPW lanes per row; the item's
// edges go in batches of SL, lane l of the slot owning edge e0 + l:
//   pass 1: the lane scores its own edge — the k row of its destination (att
//           floats, 16-byte loads) against the row's q (staged once per slot in
//           LDS, read back as broadcasts) — and the slot folds the batch into a
//           running (M_h, L_h) by xor trees (fixed order);
//   pass 2: each lane turns its edge's scores into the weight w_e (kept in
//           registers for an item of one batch, recomputed from k otherwise)
//           and K1's gather loop aggregates x with it (U edges in flight), the
//           RHS / Runge-Kutta epilogue fused as in K1.
// A lane scoring a whole edge costs att FMAs per edge against ~10 VALU per edge
// and head for a slot-cooperative score (the first version of this kernel,
// 158 us on G-arxiv against 86 us for K1, was VALU-bound that way).
//
// Hub rows (more than `chunk` edges, split into chunk items, as in K1): a chunk
// forms its own statistics and per-head unnormalised sums, which the last chunk
// of the row to arrive merges with the rescaling of the online softmax
// (dot_hub_combine; arrival tickets on the plan's heavy entries, fixed merge
// order).  A wavefront holding a chunk accumulates per head for all its rows.
// (A one-workgroup-per-hub statistics pre-pass launched first, so that chunks
// weight with final statistics and merge like K1's, measured 17 us on G-arxiv.)
#include <type_traits>

#include "aggregate.hpp"
#include "rhs_host.hpp"

namespace gnpde {

constexpr float kLog2e = 1.4426950408889634f;

// A/B knobs of variant builds (make variant VFLAGS=...; the product build uses the defaults)
#ifndef GNPDE_FL_PREFETCH
#define GNPDE_FL_PREFETCH 0  // batch 0's first U gathers issued before pass 1 (195 against 176 us: registers)
#endif
#ifndef GNPDE_FL_TILEU
#define GNPDE_FL_TILEU 4     // score-tile load instructions in flight
#endif
#ifndef GNPDE_FL_U
#define GNPDE_FL_U 4         // edges in flight per row in the gather loop
#endif
#ifndef GNPDE_FL_DIAG
#define GNPDE_FL_DIAG 0      // diagnostics only (wrong results): 1 no pass 1, 2 no pass-2 rescoring, 3 no slot reductions
#endif
#ifndef GNPDE_FL_DPPRED
#define GNPDE_FL_DPPRED 1    // slot max / sum by DPP inside 16-lane rows (+ one swizzle per further row)
#endif
#ifndef GNPDE_FL_WAVES
#define GNPDE_FL_WAVES 0     // amdgpu_waves_per_eu floor of the aggregation kernel (0: none)
#endif

struct DotArgs {
  const float* __restrict__ q;  // [R, ldqk]: q_r at q + r*ldqk, att = H*dk floats
  const float* __restrict__ k;
  int64_t ldqk;
  float scale;                  // log2(e) / sqrt(dk)
  double scale64;               // the same in fp64 (the one-pass kernel's fp64 scores)
};

// sum over the S = dk/4 lanes of a head (S in {1, 2, 4, 8, 16}, aligned inside a 16-lane row)
template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}
template <int S>
__device__ __forceinline__ float head_reduce(float v) {
  if constexpr (S >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (S >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (S >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if constexpr (S >= 16) v += dpp_mov<0x140>(v); // row_mirror
  return v;
}

// the same over fp64 values (dpp_mov64: common.hpp)
template <int S>
__device__ __forceinline__ double head_reduce64(double v) {
  if constexpr (S >= 2) v += dpp_mov64<0xB1>(v);
  if constexpr (S >= 4) v += dpp_mov64<0x4E>(v);
  if constexpr (S >= 8) v += dpp_mov64<0x141>(v);
  if constexpr (S >= 16) v += dpp_mov64<0x140>(v);
  return v;
}

// Scores of n <= SL edges (destinations mc of lanes [base, base + n)) against
// one row's q, in score tiles: NA = att/4 lanes per edge, each holding one
// 16-byte slice of q (qv) and loading the same slice of its edge's k row, so one
// load instruction covers SL/NA whole k rows (whole cache lines, no lane
// re-reading a line another load already touched); the dk/4 lanes of a head
// sum by DPP, and the head's first lane writes the score to the slot's LDS
// scores sc[e][h].  kTileU instructions' loads are in flight together.
constexpr int kTileU = GNPDE_FL_TILEU;

template <int SL, int NA, int S, int H>
__device__ __forceinline__ void tile_scores(const float (&qv)[4], int mc, int n, int base, int sl, const DotArgs& da,
                                            float* __restrict__ sc) {
  constexpr int EPI = SL / NA;  // edges per load instruction
  const int sub = sl % NA, eo = sl / NA;
  for (int i0 = 0; i0 < n; i0 += EPI * kTileU) {
    float4 kv[kTileU];
#pragma unroll
    for (int u = 0; u < kTileU; ++u) {
      const int e = i0 + u * EPI + eo;
      const int c = __shfl(mc, base + (e < SL ? e : 0));
      kv[u] = e < n ? *reinterpret_cast<const float4*>(da.k + (int64_t)c * da.ldqk + 4 * sub)
                    : make_float4(0.f, 0.f, 0.f, 0.f);
    }
#pragma unroll
    for (int u = 0; u < kTileU; ++u) {
      const int e = i0 + u * EPI + eo;
      float d = qv[0] * kv[u].x;
      d = fmaf(qv[1], kv[u].y, d);
      d = fmaf(qv[2], kv[u].z, d);
      d = fmaf(qv[3], kv[u].w, d);
      d = head_reduce<S>(d) * da.scale;  // DPP inside the NA-lane group
      if (e < n && sub % S == 0) sc[e * H + sub / S] = d;
    }
  }
}

// the lane's own edge's scores back from the slot's LDS tile (-inf past n)
template <int H>
__device__ __forceinline__ void own_scores(const float* __restrict__ sc, int sl, int n, float (&s)[H]) {
#pragma unroll
  for (int h = 0; h < H; ++h) s[h] = sl < n ? sc[sl * H + h] : -INFINITY;
}

// xor trees over the SL lanes of a row slot (SL a power of two, slots aligned)
template <int SL>
__device__ __forceinline__ float slot_max(float v) {
  if constexpr (GNPDE_FL_DPPRED) {
    v = fmaxf(v, dpp_mov<0xB1>(v));
    v = fmaxf(v, dpp_mov<0x4E>(v));
    v = fmaxf(v, dpp_mov<0x141>(v));
    v = fmaxf(v, dpp_mov<0x140>(v));
#pragma unroll
    for (int o = 16; o < SL; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
    return v;
  }
#pragma unroll
  for (int o = 1; o < SL; o <<= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
template <int SL>
__device__ __forceinline__ float slot_sum(float v) {
  if constexpr (GNPDE_FL_DPPRED) {
    v += dpp_mov<0xB1>(v);
    v += dpp_mov<0x4E>(v);
    v += dpp_mov<0x141>(v);
    v += dpp_mov<0x140>(v);
#pragma unroll
    for (int o = 16; o < SL; o <<= 1) v += __shfl_xor(v, o);
    return v;
  }
#pragma unroll
  for (int o = 1; o < SL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// the edge weight from its scores and the group statistics (M, Rl = 1/(L + eps))
template <int H>
__device__ __forceinline__ float edge_weight(const float (&s)[H], const float (&M)[H], const float (&Rl)[H]) {
  float w = 0.f;
#pragma unroll
  for (int h = 0; h < H; ++h) w = fmaf(__builtin_amdgcn_exp2f(s[h] - M[h]), Rl[h], w);
  constexpr float inv_h = 1.0f / (float)H;
  return w * inv_h;
}

// ------------------------------------------------------------------ hub rows
// A chunk of a hub row keeps its own statistics: per head the chunk max M_c,
// sum L_c and the unnormalised sum acc_c = sum_e exp(s_e - M_c) x_e, stored
// write-through in its partial slot ([H][C] acc, then M[H], L[H]; ps floats).
// The last chunk to arrive merges the slots in chunk order:
//   M = max_c M_c,  L = sum_c L_c 2^(M_c - M),  acc = sum_c acc_c 2^(M_c - M)
// and runs the epilogue with ax = (1/H) sum_h acc_h / (L_h + 1e-16).  Lanes cover
// the columns (C <= 256: 4 per lane).
__host__ __device__ constexpr int64_t dot_partial_floats(int64_t H, int64_t C) { return (H * C + 2 * H + 3) & ~3; }

template <int H, int STG, class T = float>
__device__ __forceinline__ void dot_hub_combine(int row, int first, int nch, int C, int ps, const Epi& ep,
                                                const float* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int cc = lane * 4;
  const bool live = cc < C;
  float M[H], L[H], acc[H][4];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = 0.f;
  }
  for (int c = 0; c < nch; ++c) {
    const float* p = partials + (int64_t)(first + c) * ps;
#pragma unroll
    for (int h = 0; h < H; ++h) M[h] = fmaxf(M[h], p[H * C + h]);
  }
  for (int c = 0; c < nch; ++c) {
    const float* p = partials + (int64_t)(first + c) * ps;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float f = __builtin_amdgcn_exp2f(p[H * C + h] - M[h]);
      L[h] = fmaf(p[H * C + H + h], f, L[h]);
      if (live) {
        float v[4];
        load_vec<4>(p + h * C + cc, v);
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[h][t] = fmaf(v[t], f, acc[h][t]);
      }
    }
  }
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float r = 1.0f / (L[h] + kSoftmaxEps);
#pragma unroll
    for (int t = 0; t < 4; ++t) ax[t] = fmaf(acc[h][t], r, ax[t]);
  }
  constexpr float inv_h = 1.0f / (float)H;
#pragma unroll
  for (int t = 0; t < 4; ++t) ax[t] *= inv_h;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (live) epilogue_store<4, STG, T>(ep, row, cc, ax, a, b, &dpart);
  static_assert(!stage_dot<STG>(), "dot-term epilogues are not fused here");
}

// ------------------------------------------------------------------ the fused attention RHS
template <int GL, int U, int NA, int S, int H, int STG>
__global__ __launch_bounds__(256)
#if GNPDE_FL_WAVES
__attribute__((amdgpu_waves_per_eu(GNPDE_FL_WAVES)))
#endif
void dot_agg_kernel(const int4* __restrict__ items, int n_items, int4* heavy, int n_heavy,
                    const int* __restrict__ col, DotArgs da, int C, Epi ep, float* __restrict__ partials) {
  constexpr int RPW = kWave / GL;
  constexpr int SL = GL;
  __shared__ float scs[kWavesPerBlock][RPW][SL * H];  // each slot's batch scores
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rs = lane / SL, sl = lane % SL;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + wv);
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const int cc = sl * 4;
  const bool owner = live && slot < 0 && cc < C;
  const bool chunk = live && slot >= 0;
  const int base = rs * SL;
  float* sc = scs[wv][rs];
  // a wavefront holding a hub chunk accumulates per head (its statistics are the chunk's own)
  int wchunk = 0;
  if (n_heavy > 0) {
#pragma unroll
    for (int r = 0; r < RPW; ++r) wchunk |= __shfl((int)chunk, r * SL);
  }
  wchunk = uniform(wchunk);

  EpiPre<4, float, STG> pre;
  if (owner) epi_prefetch<4, STG, float>(ep, row, cc, pre);
  float qv[4];  // this lane's slice of the row's q (score tiles)
  load_vec<4>(da.q + (int64_t)row * da.ldqk + 4 * (sl % NA), qv);

  const int len = end - beg;
  const int mc0 = sl < len ? col[beg + sl] : 0;
  // batch 0's first U gathers issued before pass 1 (A/B knob; off: the registers cost more)
  float xv0[U][4];
#pragma unroll
  for (int u = 0; u < (GNPDE_FL_PREFETCH ? U : 0); ++u) {
    const int c = __shfl(mc0, base + (u < len ? u : 0));
    if (u < len && cc < C) {
      load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, xv0[u]);
    } else {
#pragma unroll
      for (int t = 0; t < 4; ++t) xv0[u][t] = 0.f;
    }
  }
  float M[H], L[H], Rl[H];
  float s1[H];  // the lane's scores of batch 0 (kept for pass 2)
#pragma unroll
  for (int h = 0; h < H; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
  }
  // pass 1: the statistics of the item's edges, batch by batch
  for (int e0 = 0; e0 < (GNPDE_FL_DIAG == 1 ? 0 : len); e0 += SL) {
    const int n = min(SL, len - e0);
    const int mc = e0 == 0 ? mc0 : (sl < n ? col[beg + e0 + sl] : 0);
    tile_scores<SL, NA, S, H>(qv, mc, n, base, sl, da, sc);
    float s[H];
    own_scores<H>(sc, sl, n, s);
    if (e0 == 0) {
#pragma unroll
      for (int h = 0; h < H; ++h) s1[h] = s[h];
    }
    if (GNPDE_FL_DIAG == 3) break;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      const float mb = slot_max<SL>(s[h]);  // inside the slot (slot-uniform control flow)
      const float mn = fmaxf(M[h], mb);
      const float lb = slot_sum<SL>(__builtin_amdgcn_exp2f(s[h] - mn));  // s = -inf -> 0
      L[h] = fmaf(L[h], __builtin_amdgcn_exp2f(M[h] - mn), lb);
      M[h] = mn;
    }
  }
#pragma unroll
  for (int h = 0; h < H; ++h) Rl[h] = 1.0f / (L[h] + kSoftmaxEps);

  // pass 2: K1's gather loop; one finished weight per edge, or (a wavefront with a
  // hub chunk) one unnormalised weight per edge and head.  The two forms are separate
  // branches with their own accumulators, so the per-head sums of the chunk form
  // hold no registers in the whole-row form (114 -> fewer VGPRs, more waves).
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  if (!wchunk) {
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int e0 = 0; e0 < len; e0 += SL) {
      const int n = min(SL, len - e0);
      int mc;
      float s[H];
      if (e0 == 0 || GNPDE_FL_DIAG) {
        mc = e0 == 0 ? mc0 : (sl < n ? col[beg + e0 + sl] : 0);
#pragma unroll
        for (int h = 0; h < H; ++h) s[h] = GNPDE_FL_DIAG == 1 ? 0.f : s1[h];
      } else {  // a later batch of a long row: its scores again
        mc = sl < n ? col[beg + e0 + sl] : 0;
        tile_scores<SL, NA, S, H>(qv, mc, n, base, sl, da, sc);
        own_scores<H>(sc, sl, n, s);
      }
      const float mw = sl < n ? edge_weight<H>(s, M, Rl) : 0.f;
      for (int j = 0; j < n; j += U) {
        float v[U][4];
        float ww[U];
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const int jj = j + u;
          const int src = base + (jj < n ? jj : 0);
          const int c = __shfl(mc, src);
          ww[u] = jj < n ? __shfl(mw, src) : 0.f;
          if (GNPDE_FL_PREFETCH && e0 == 0 && j == 0) {  // gathered before pass 1
#pragma unroll
            for (int t = 0; t < 4; ++t) v[u][t] = xv0[u][t];
          } else if (jj < n && cc < C) {
            load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, v[u]);
          } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) v[u][t] = 0.f;
          }
        }
#pragma unroll
        for (int u = 0; u < U; ++u)
#pragma unroll
          for (int t = 0; t < 4; ++t) acc[t] = fmaf(ww[u], v[u][t], acc[t]);
      }
    }
    if (!live) return;
    double dpart = 0.0;
    if (owner) epi_finish<4, STG, float>(ep, row, cc, acc, a, b, pre, &dpart);
    (void)dpart;
    return;
  }
  // hub-chunk wavefronts gather UC rows at a time: their per-head weights and sums
  // would otherwise set the kernel's register count
  constexpr int UC = U > 2 ? U / 2 : U;
  float acch[H][4];
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int t = 0; t < 4; ++t) acch[h][t] = 0.f;
  for (int e0 = 0; e0 < len; e0 += SL) {
    const int n = min(SL, len - e0);
    int mc;
    float s[H];
    if (e0 == 0 || GNPDE_FL_DIAG) {
      mc = e0 == 0 ? mc0 : (sl < n ? col[beg + e0 + sl] : 0);
#pragma unroll
      for (int h = 0; h < H; ++h) s[h] = GNPDE_FL_DIAG == 1 ? 0.f : s1[h];
    } else {
      mc = sl < n ? col[beg + e0 + sl] : 0;
      tile_scores<SL, NA, S, H>(qv, mc, n, base, sl, da, sc);
      own_scores<H>(sc, sl, n, s);
    }
    float ph[H];
#pragma unroll
    for (int h = 0; h < H; ++h) ph[h] = sl < n ? __builtin_amdgcn_exp2f(s[h] - M[h]) : 0.f;
    for (int j = 0; j < n; j += UC) {
      float v[UC][4];
      float ww[UC][H];
#pragma unroll
      for (int u = 0; u < UC; ++u) {
        const int jj = j + u;
        const int src = base + (jj < n ? jj : 0);
        const int c = __shfl(mc, src);
#pragma unroll
        for (int h = 0; h < H; ++h) ww[u][h] = jj < n ? __shfl(ph[h], src) : 0.f;
        if (GNPDE_FL_PREFETCH && e0 == 0 && j < U) {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[u][t] = xv0[(j + u) % U][t];
        } else if (jj < n && cc < C) {
          load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, v[u]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[u][t] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < UC; ++u)
#pragma unroll
        for (int h = 0; h < H; ++h)
#pragma unroll
          for (int t = 0; t < 4; ++t) acch[h][t] = fmaf(ww[u][h], v[u][t], acch[h][t]);
    }
  }
  {
    // hub chunks: (acc_h, M_h, L_h) written through to the slot, merged in-launch by
    // the last arrival (arrival tickets on the plan's heavy entries, as K1)
    const int ps = (int)dot_partial_floats(H, C);
    const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
    const int64_t pb = (int64_t)(chunk ? slot : 0) * ps;
#pragma unroll
    for (int h = 0; h < H; ++h) {
      buf_store_wt<4>(rp, (chunk && cc < C) ? (uint32_t)((pb + h * C + cc) * 4) : kBufNone, acch[h]);
      float ml[1] = {M[h]};
      buf_store_wt<1>(rp, (chunk && sl == 0) ? (uint32_t)((pb + H * C + h) * 4) : kBufNone, ml);
      ml[0] = L[h];
      buf_store_wt<1>(rp, (chunk && sl == 0) ? (uint32_t)((pb + H * C + H + h) * 4) : kBufNone, ml);
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    int lo = 0, won = 0;
    if (chunk) {
      int hi = n_heavy - 1;
      while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (heavy[mid].y <= slot)
          lo = mid;
        else
          hi = mid - 1;
      }
      if (sl == 0) {
        const int t = __hip_atomic_fetch_add(&heavy[lo].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
        won = t == heavy[lo].z - 1;
      }
    }
#pragma unroll
    for (int r = 0; r < RPW; ++r) {
      if (__shfl(won, r * SL)) {  // wave-uniform
        const int hh = __shfl(lo, r * SL);
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
        const int4 hv = heavy[hh];
        dot_hub_combine<H, STG>(uniform(hv.x), uniform(hv.y), uniform(hv.z), C, ps, ep, partials);
        if (lane == 0) __hip_atomic_store(&heavy[hh].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      }
    }
  }
  if (chunk) return;
  // the whole rows of this wavefront: normalise the per-head sums
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < H; ++h)
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = fmaf(acch[h][t], Rl[h], acc[t]);
  constexpr float inv_h = 1.0f / (float)H;
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] *= inv_h;
  if (!live) return;
  double dpart = 0.0;
  if (owner) epi_finish<4, STG, float>(ep, row, cc, acc, a, b, pre, &dpart);
  (void)dpart;
}

// ------------------------------------------------------------------ the one-pass form (round 4)
// The same RHS in ONE pass over the item's edges, the online softmax of
// flash attention per head: each batch of U edges of a row slot gathers the
// edges' x rows AND k rows together (one memory latency per batch, not one for
// the scores and another for the rows).  The k rows go through score tiles as in
// tile_scores (NA = att/4 lanes per edge, 16-byte slices, EPI = SL/NA edges per
// load; the same four fmas and DPP head sums, so the same score bits as the
// two-pass kernel), the head scores are broadcast to the slot, and each head
// keeps a running (M_h, L_h, acc_h = sum_e 2^(s_e,h - M_h) x_e), rescaled by
// 2^(M_old - M_new) once per batch.  The row's result is
//   ax = (1/H) sum_h acc_h / (L_h + 1e-16)
// — the two-pass kernel's sum, each head's exponentials taken against the
// running rather than the final max (same value up to rounding).  Hub chunks
// write their (acc_h, M_h rounded to fp32, L_h) and merge exactly as above
// (dot_hub_combine).  G-arxiv per-edge RHS (norm_idx 0): 0.171 -> 0.151 ms.
#ifndef GNPDE_FL_ONEPASS
#define GNPDE_FL_ONEPASS 1   // A/B: 0 keeps the two-pass kernel above
#endif
#ifndef GNPDE_FL_SCORE64
#define GNPDE_FL_SCORE64 0   // A/B: 1 head sums, scores and the running max in fp64 (0.202 against 0.151 ms)
#endif
using ScoreT = std::conditional_t<GNPDE_FL_SCORE64 != 0, double, float>;

template <int GL, int U, int ATT, int H, int STG, class T = float>
__global__ __launch_bounds__(256) void dot_agg1_kernel(const int4* __restrict__ items, int n_items, int4* heavy,
                                                        int n_heavy, const int* __restrict__ col, DotArgs da, int C,
                                                        Epi ep, float* __restrict__ partials) {
  constexpr int RPW = kWave / GL;
  constexpr int SL = GL;
  constexpr int NA = ATT / 4;                  // lanes per edge of a score tile (16-byte slices)
  constexpr int S = NA / H;                    // lanes per head
  constexpr int EPI = SL / NA;                 // edges per tile load
  constexpr int TL = (U + EPI - 1) / EPI;      // tile loads per batch of U edges
  static_assert(NA <= SL && S >= 1 && S <= 16 && (S & (S - 1)) == 0, "dot_agg1: score tile layout");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rs = lane / SL, sl = lane % SL;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + wv);
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const int cc = sl * 4;
  const bool owner = live && slot < 0 && cc < C;
  const bool chunk = live && slot >= 0;
  const int base = rs * SL;
  const int sub = sl % NA, eo = sl / NA;

  EpiPre<4, T, STG> pre;
  if (owner) epi_prefetch<4, STG, T>(ep, row, cc, pre);
  float qv[4];  // this lane's slice of the row's q (score tiles, as tile_scores)
  load_vec<4>(da.q + (int64_t)row * da.ldqk + 4 * sub, qv);

  ScoreT M[H];
  float L[H], acch[H][4];
#pragma unroll
  for (int h = 0; h < H; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acch[h][t] = 0.f;
  }
  const int len = end - beg;
  for (int e0 = 0; e0 < len; e0 += SL) {
    const int n = min(SL, len - e0);
    const int mc = sl < n ? col[beg + e0 + sl] : 0;
    for (int j = 0; j < n; j += U) {
      float v[U][4], kt[TL][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u;
        const int c = __shfl(mc, base + (jj < n ? jj : 0));
        if (jj < n && cc < C) {
          if constexpr (sizeof(T) == 4) {
            load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, v[u]);
          } else {  // bf16 state: 8-byte row slices, widened in registers
            Packed<4, T> pk;
            load_packed<4>(as_t<T>(ep.x) + (int64_t)c * ep.ldx + cc, pk);
#pragma unroll
            for (int t = 0; t < 4; ++t) v[u][t] = unpack(pk, t);
          }
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[u][t] = 0.f;
        }
      }
      // score tiles: lane (eo, sub) loads the 16-byte slice sub of edge g*EPI + eo's k row
#pragma unroll
      for (int g = 0; g < TL; ++g) {
        const int ue = g * EPI + eo;  // the batch edge of this lane's tile slot
        const int jj = j + ue;
        const int c = __shfl(mc, base + (jj < n ? jj : 0));
        if (ue < U && jj < n) {
          load_vec<4>(da.k + (int64_t)c * da.ldqk + 4 * sub, kt[g]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) kt[g][t] = 0.f;
        }
      }
      // the scores, summed exactly as tile_scores (four fmas, then the head's lanes by DPP)
      ScoreT dt[TL];
#pragma unroll
      for (int g = 0; g < TL; ++g) {
        float d = qv[0] * kt[g][0];
        d = fmaf(qv[1], kt[g][1], d);
        d = fmaf(qv[2], kt[g][2], d);
        d = fmaf(qv[3], kt[g][3], d);
        if constexpr (GNPDE_FL_SCORE64)
          dt[g] = head_reduce64<S>((double)d) * da.scale64;
        else
          dt[g] = head_reduce<S>(d) * da.scale;
      }
      ScoreT sc[U][H];
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const ScoreT x = __shfl(dt[u / EPI], base + (u % EPI) * NA + h * S);
          sc[u][h] = j + u < n ? x : -INFINITY;
        }
#pragma unroll
      for (int h = 0; h < H; ++h) {
        ScoreT mb = M[h];
#pragma unroll
        for (int u = 0; u < U; ++u) mb = fmax(mb, sc[u][h]);
        const float r = __builtin_amdgcn_exp2f((float)(M[h] - mb));  // M = -inf: 0 (the sums are 0 too)
        L[h] *= r;
#pragma unroll
        for (int t = 0; t < 4; ++t) acch[h][t] *= r;
#pragma unroll
        for (int u = 0; u < U; ++u) {
          const float pw = __builtin_amdgcn_exp2f((float)(sc[u][h] - mb));  // -inf past n: 0
          L[h] += pw;
#pragma unroll
          for (int t = 0; t < 4; ++t) acch[h][t] = fmaf(pw, v[u][t], acch[h][t]);
        }
        M[h] = mb;
      }
    }
  }
  if (n_heavy > 0) {
    int anyc = 0;
#pragma unroll
    for (int r = 0; r < RPW; ++r) anyc |= __shfl((int)chunk, r * SL);
    if (anyc) {  // wave-uniform: hub chunks write (acc_h, M_h, L_h) through; the last arrival merges
      const int ps = (int)dot_partial_floats(H, C);
      const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
      const int64_t pb = (int64_t)(chunk ? slot : 0) * ps;
#pragma unroll
      for (int h = 0; h < H; ++h) {
        // the slot keeps the max rounded to fp32, the sums taken relative to it
        const float mf = (float)M[h];
        const float adj = __builtin_amdgcn_exp2f((float)(M[h] - (double)mf));
        float av[4];
#pragma unroll
        for (int t = 0; t < 4; ++t) av[t] = acch[h][t] * adj;
        buf_store_wt<4>(rp, (chunk && cc < C) ? (uint32_t)((pb + h * C + cc) * 4) : kBufNone, av);
        float ml[1] = {mf};
        buf_store_wt<1>(rp, (chunk && sl == 0) ? (uint32_t)((pb + H * C + h) * 4) : kBufNone, ml);
        ml[0] = L[h] * adj;
        buf_store_wt<1>(rp, (chunk && sl == 0) ? (uint32_t)((pb + H * C + H + h) * 4) : kBufNone, ml);
      }
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      int lo = 0, won = 0;
      if (chunk) {
        int hi = n_heavy - 1;
        while (lo < hi) {
          const int mid = (lo + hi + 1) >> 1;
          if (heavy[mid].y <= slot)
            lo = mid;
          else
            hi = mid - 1;
        }
        if (sl == 0) {
          const int t = __hip_atomic_fetch_add(&heavy[lo].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
          won = t == heavy[lo].z - 1;
        }
      }
#pragma unroll
      for (int r = 0; r < RPW; ++r) {
        if (__shfl(won, r * SL)) {  // wave-uniform
          const int hh = __shfl(lo, r * SL);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          const int4 hv = heavy[hh];
          dot_hub_combine<H, STG, T>(uniform(hv.x), uniform(hv.y), uniform(hv.z), C, ps, ep, partials);
          if (lane == 0) __hip_atomic_store(&heavy[hh].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
    }
  }
  if (!live || chunk) return;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < H; ++h) {
    const float rl = 1.0f / (L[h] + kSoftmaxEps);
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[t] = fmaf(acch[h][t], rl, acc[t]);
  }
  constexpr float inv_h = 1.0f / (float)H;
#pragma unroll
  for (int t = 0; t < 4; ++t) acc[t] *= inv_h;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (owner) epi_finish<4, STG, T>(ep, row, cc, acc, a, b, pre, &dpart);
  (void)dpart;
}

// ------------------------------------------------------------------ per-edge scores, destination-grouped softmax
// attention_norm_idx 1: the softmax group of an edge is its destination, so its
// statistics come from the CSC statistics kernel (gnpde_seg_softmax_f32 -> the
// packed records {m[h], rl[h]} of every destination) and this pass only scores
// the edges it gathers (score tiles, as above) and weights them:
//   w_e = (1/H) sum_h exp(s_e,h - m[c,h]) * rl[c,h]
// — the weights pass (gnpde_attn_weights_f32) and its [nnz] round trip fused into
// K1; hub chunks merge exactly like K1's (the weights are final).
template <int GL, int U, int NA, int S, int H, int STG>
__global__ __launch_bounds__(256) void dot_dst_agg_kernel(const int4* __restrict__ items, int n_items, int4* heavy,
                                                           int n_heavy, const int* __restrict__ col, DotArgs da,
                                                           const float* __restrict__ rec, int C, Epi ep,
                                                           float* __restrict__ partials) {
  constexpr int RPW = kWave / GL;
  constexpr int SL = GL;
  constexpr int RF = stats_record_floats(H);
  __shared__ float scs[kWavesPerBlock][RPW][SL * H];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rs = lane / SL, sl = lane % SL;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + wv);
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const int cc = sl * 4;
  const bool owner = live && slot < 0 && cc < C;
  const int base = rs * SL;
  float* sc = scs[wv][rs];

  EpiPre<4, float, STG> pre;
  if (owner) epi_prefetch<4, STG, float>(ep, row, cc, pre);
  float qv[4];
  load_vec<4>(da.q + (int64_t)row * da.ldqk + 4 * (sl % NA), qv);
  const int len = end - beg;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e0 = 0; e0 < len; e0 += SL) {
    const int n = min(SL, len - e0);
    const int mc = sl < n ? col[beg + e0 + sl] : 0;
    // the destination's record, issued with the score tile's loads
    float rm[H], rr[H];
    if constexpr (RF == 4 && H == 2) {
      const float4 v = *reinterpret_cast<const float4*>(rec + (int64_t)mc * 4);
      rm[0] = v.x; rm[1] = v.y; rr[0] = v.z; rr[1] = v.w;
    } else {
#pragma unroll
      for (int h = 0; h < H; ++h) {
        rm[h] = rec[(int64_t)mc * RF + h];
        rr[h] = rec[(int64_t)mc * RF + H + h];
      }
    }
    tile_scores<SL, NA, S, H>(qv, mc, n, base, sl, da, sc);
    float s[H];
    own_scores<H>(sc, sl, n, s);
    float mw = 0.f;
    if (sl < n) {
#pragma unroll
      for (int h = 0; h < H; ++h) mw = fmaf(__builtin_amdgcn_exp2f(s[h] - rm[h] * kLog2e), rr[h], mw);
      constexpr float inv_h = 1.0f / (float)H;
      mw *= inv_h;
    }
    for (int j = 0; j < n; j += U) {
      float v[U][4];
      float ww[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u;
        const int src = base + (jj < n ? jj : 0);
        const int c = __shfl(mc, src);
        ww[u] = jj < n ? __shfl(mw, src) : 0.f;
        if (jj < n && cc < C) {
          load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, v[u]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[u][t] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = fmaf(ww[u], v[u][t], acc[t]);
    }
  }
  if (n_heavy > 0) {  // hub chunks: write-through partials, merged in-launch by the last arrival (K1's)
    const bool chunk = live && slot >= 0;
    int anyc = 0;
#pragma unroll
    for (int r = 0; r < RPW; ++r) anyc |= __shfl((int)chunk, r * SL);
    if (anyc) {  // wave-uniform
      const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
      buf_store_wt<4>(rp, (chunk && cc < C) ? (uint32_t)(((int64_t)slot * C + cc) * 4) : kBufNone, acc);
      hub_arrive_slots<4, GL, SL, RPW, STG, float>(heavy, n_heavy, chunk, slot, C, ep, partials);
      if (chunk) return;
    }
  }
  if (!live || slot >= 0) return;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (owner) epi_finish<4, STG, float>(ep, row, cc, acc, a, b, pre, &dpart);
  (void)dpart;
}

// The one-pass form of the destination-grouped kernel (round 4, A/B knob
// GNPDE_FL_DST1, off): each batch of U edges gathers the edges' x rows, their
// k-row score tiles and their statistics records together, then weights and
// accumulates (as dot_agg1_kernel; the score bits are those of tile_scores).
// Measured: per-edge norm_idx 1 RHS 0.1706 against 0.1731 ms in the solve's
// numbering, 0.1938 against 0.1851 in the user numbering (the per-batch record
// loads) — not taken.
#ifndef GNPDE_FL_DST1
#define GNPDE_FL_DST1 0
#endif
template <int GL, int U, int ATT, int H, int STG>
__global__ __launch_bounds__(256) void dot_dst_agg1_kernel(const int4* __restrict__ items, int n_items, int4* heavy,
                                                            int n_heavy, const int* __restrict__ col, DotArgs da,
                                                            const float* __restrict__ rec, int C, Epi ep,
                                                            float* __restrict__ partials) {
  constexpr int RPW = kWave / GL;
  constexpr int SL = GL;
  constexpr int RF = stats_record_floats(H);
  constexpr int NA = ATT / 4;
  constexpr int S = NA / H;
  constexpr int EPI = SL / NA;
  constexpr int TL = (U + EPI - 1) / EPI;
  static_assert(NA <= SL && S >= 1 && S <= 16 && (S & (S - 1)) == 0, "dot_dst_agg1: score tile layout");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int rs = lane / SL, sl = lane % SL;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + wv);
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const int cc = sl * 4;
  const bool owner = live && slot < 0 && cc < C;
  const int base = rs * SL;
  const int sub = sl % NA, eo = sl / NA;

  EpiPre<4, float, STG> pre;
  if (owner) epi_prefetch<4, STG, float>(ep, row, cc, pre);
  float qv[4];
  load_vec<4>(da.q + (int64_t)row * da.ldqk + 4 * sub, qv);
  const int len = end - beg;
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  for (int e0 = 0; e0 < len; e0 += SL) {
    const int n = min(SL, len - e0);
    const int mc = sl < n ? col[beg + e0 + sl] : 0;
    for (int j = 0; j < n; j += U) {
      float v[U][4], kt[TL][4], rm[U][H], rr[U][H];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u;
        const int c = __shfl(mc, base + (jj < n ? jj : 0));
        if (jj < n && cc < C) {
          load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, v[u]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) v[u][t] = 0.f;
        }
        // the destination's statistics record (one line; the same address across the slot)
        if constexpr (RF == 4 && H == 2) {
          const float4 r4 = *reinterpret_cast<const float4*>(rec + (int64_t)c * 4);
          rm[u][0] = r4.x; rm[u][1] = r4.y; rr[u][0] = r4.z; rr[u][1] = r4.w;
        } else {
#pragma unroll
          for (int h = 0; h < H; ++h) {
            rm[u][h] = rec[(int64_t)c * RF + h];
            rr[u][h] = rec[(int64_t)c * RF + H + h];
          }
        }
      }
#pragma unroll
      for (int g = 0; g < TL; ++g) {
        const int ue = g * EPI + eo;
        const int jj = j + ue;
        const int c = __shfl(mc, base + (jj < n ? jj : 0));
        if (ue < U && jj < n) {
          load_vec<4>(da.k + (int64_t)c * da.ldqk + 4 * sub, kt[g]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) kt[g][t] = 0.f;
        }
      }
      float dt[TL];
#pragma unroll
      for (int g = 0; g < TL; ++g) {
        float d = qv[0] * kt[g][0];
        d = fmaf(qv[1], kt[g][1], d);
        d = fmaf(qv[2], kt[g][2], d);
        d = fmaf(qv[3], kt[g][3], d);
        dt[g] = head_reduce<S>(d) * da.scale;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float w = 0.f;
#pragma unroll
        for (int h = 0; h < H; ++h) {
          const float sh = __shfl(dt[u / EPI], base + (u % EPI) * NA + h * S);
          w = fmaf(__builtin_amdgcn_exp2f(sh - rm[u][h] * kLog2e), rr[u][h], w);
        }
        constexpr float inv_h = 1.0f / (float)H;
        w = j + u < n ? w * inv_h : 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) acc[t] = fmaf(w, v[u][t], acc[t]);
      }
    }
  }
  if (n_heavy > 0) {  // hub chunks: write-through partials, merged in-launch by the last arrival (K1's)
    const bool chunk = live && slot >= 0;
    int anyc = 0;
#pragma unroll
    for (int r = 0; r < RPW; ++r) anyc |= __shfl((int)chunk, r * SL);
    if (anyc) {  // wave-uniform
      const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
      buf_store_wt<4>(rp, (chunk && cc < C) ? (uint32_t)(((int64_t)slot * C + cc) * 4) : kBufNone, acc);
      hub_arrive_slots<4, GL, SL, RPW, STG, float>(heavy, n_heavy, chunk, slot, C, ep, partials);
      if (chunk) return;
    }
  }
  if (!live || slot >= 0) return;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (owner) epi_finish<4, STG, float>(ep, row, cc, acc, a, b, pre, &dpart);
  (void)dpart;
}

template <int GL, int NA, int S, int H, class T = float>
static int launch_dot_nh(const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                         const DotArgs& da, const float* rec, int C, const Epi& ep, float* partials, hipStream_t s) {
  constexpr int RPW = kWave / GL;
  constexpr int U = GNPDE_FL_U;
  const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * RPW);
  const int stg = epi_stage_kind(ep);
  const int nh = (int)n_heavy;
  if constexpr (sizeof(T) != 4) {
    // a bf16 state: the one-pass source-grouped kernel only (the caller takes K2 + the bf16 K1 otherwise)
    if (rec != nullptr || stg >= 2 || !(GNPDE_FL_ONEPASS && NA <= GL)) {
      set_error("attn_dot_rhs_bf16: only the source-grouped plain RHS and single-output stages are fused");
      return GNPDE_EUNSUPPORTED;
    }
    if (stg == 1)
      dot_agg1_kernel<GL, U, 4 * NA, H, 1, T><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep,
                                                                      partials);
    else
      dot_agg1_kernel<GL, U, 4 * NA, H, 0, T><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep,
                                                                      partials);
    GNPDE_LAUNCH_CHECK();
    return GNPDE_OK;
  }
  if (rec != nullptr) {  // destination-grouped softmax (norm_idx 1): statistics records given
    if constexpr (GNPDE_FL_DST1 && 4 * NA <= 4 * GL) {
      if (stg <= 1) {
        if (stg == 1)
          dot_dst_agg1_kernel<GL, U, 4 * NA, H, 1><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da,
                                                                            rec, C, ep, partials);
        else
          dot_dst_agg1_kernel<GL, U, 4 * NA, H, 0><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da,
                                                                            rec, C, ep, partials);
        GNPDE_LAUNCH_CHECK();
        return GNPDE_OK;
      }
    }
    if (stg == 1)
      dot_dst_agg_kernel<GL, U, NA, S, H, 1><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, rec, C,
                                                                      ep, partials);
    else if (stg >= 2) {
      set_error("attn_dot_rhs: only the plain RHS and single-output stage epilogues are fused");
      return GNPDE_EUNSUPPORTED;
    } else
      dot_dst_agg_kernel<GL, U, NA, S, H, 0><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, rec, C,
                                                                      ep, partials);
    GNPDE_LAUNCH_CHECK();
    return GNPDE_OK;
  }
  constexpr int ATT = 4 * NA;
  if constexpr (GNPDE_FL_ONEPASS && NA <= GL) {
    if (stg == 1)
      dot_agg1_kernel<GL, U, ATT, H, 1><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep,
                                                                 partials);
    else if (stg == 0)
      dot_agg1_kernel<GL, U, ATT, H, 0><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep,
                                                                 partials);
    if (stg <= 1) {
      GNPDE_LAUNCH_CHECK();
      return GNPDE_OK;
    }
  }
  if (stg == 1)
    dot_agg_kernel<GL, U, NA, S, H, 1><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep, partials);
  else if (stg >= 2) {
    // two-output / dot-term stage epilogues (not used by the forward integrator): the caller
    // takes the unfused path (gnpde_seg_softmax_f32 + gnpde_spmm_rhs_f32)
    set_error("attn_dot_rhs: only the plain RHS and single-output stage epilogues are fused");
    return GNPDE_EUNSUPPORTED;
  } else
    dot_agg_kernel<GL, U, NA, S, H, 0><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep, partials);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

// (att/4, heads) pairs: att in {8, 16, 32, 64}, heads in {1, 2, 4} dividing att/4
template <int GL, class T = float>
static int launch_dot(int NA, int H, const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                      const DotArgs& da, const float* rec, int C, const Epi& ep, float* partials, hipStream_t s) {
#define GNPDE_DOT(A, HH) \
  if (NA == A && H == HH) \
    return launch_dot_nh<GL, A, (A / HH), HH, T>(items, n_items, heavy, n_heavy, col, da, rec, C, ep, partials, s)
  GNPDE_DOT(2, 1); GNPDE_DOT(2, 2);
  GNPDE_DOT(4, 1); GNPDE_DOT(4, 2); GNPDE_DOT(4, 4);
  GNPDE_DOT(8, 1); GNPDE_DOT(8, 2); GNPDE_DOT(8, 4);
  GNPDE_DOT(16, 1); GNPDE_DOT(16, 2); GNPDE_DOT(16, 4);
#undef GNPDE_DOT
  set_error("attn_dot_rhs: att=%d heads=%d not instantiated", 4 * NA, H);
  return GNPDE_EUNSUPPORTED;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_attn_dot_supported(int64_t heads, int64_t dk, int64_t C) {
  const int64_t att = heads * dk;
  if (!(heads == 1 || heads == 2 || heads == 4) || dk < 4 || dk % 4) return 0;
  if (!(att == 8 || att == 16 || att == 32 || att == 64)) return 0;
  return C >= 1 && C <= 256 && C % 4 == 0;
}

int64_t gnpde_attn_dot_workspace_floats(int64_t heads, int64_t C, int64_t n_slots) {
  return n_slots * dot_partial_floats(heads, C);
}

}  // extern "C"

// the fp32 entry and its bf16-state twin (x, x0, f and the stage rows bf16; q, k, the
// statistics and the partials fp32): 16-byte rows of fp32, 8-byte slices of bf16
template <class T>
static int attn_dot_rhs_impl(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                             const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads,
                             int64_t dk, const float* dst_stats, int64_t C, const float* x, int64_t ldx,
                             const float* x0, int64_t ldx0, const float* alpha, const float* beta, int flags, float* f,
                             int64_t ldf, float* workspace, int64_t n_slots, const gnpde_stage_epilogue_t* stage,
                             void* stream) {
  auto rows_ok = [](const void* p) { return sizeof(T) == 4 ? aligned16(p) : aligned8(p); };
  GNPDE_REQUIRE(gnpde_attn_dot_supported(heads, dk, C), GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: heads=%lld dk=%lld C=%lld outside the fused kernel (heads in {1, 2, 4}, dk %% 4 == 0, "
                "heads*dk in {8, 16, 32, 64}, C %% 4 == 0, C <= 256)",
                (long long)heads, (long long)dk, (long long)C);
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf, stage);
  int rc = check_epi(ep, C, n_heavy, workspace, n_slots);
  if (rc) return rc;
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0 && n_heavy < INT32_MAX, GNPDE_EINVAL,
                "attn_dot_rhs: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && q && k), GNPDE_EINVAL, "attn_dot_rhs: NULL plan/col/q/k");
  GNPDE_REQUIRE(n_heavy == 0 || (heavy && workspace && n_slots > 0), GNPDE_EINVAL,
                "attn_dot_rhs: hub rows need heavy and the workspace");
  GNPDE_REQUIRE(n_slots * dot_partial_floats(heads, C) * 4 < (int64_t)kBufRecords, GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: %lld partial slots exceed the 4 GiB of 32-bit buffer offsets", (long long)n_slots);
  GNPDE_REQUIRE(!dst_stats || aligned16(dst_stats), GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: the statistics records must be 16-byte aligned");
  GNPDE_REQUIRE(ldqk >= heads * dk && ldqk % 4 == 0 && aligned16(q) && aligned16(k), GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: q/k rows must be 16-byte aligned (ldqk %% 4 == 0)");
  GNPDE_REQUIRE(ldx % 4 == 0 && ldf % 4 == 0 && rows_ok(x) && (!f || rows_ok(f)) && aligned16(workspace),
                GNPDE_EUNSUPPORTED, "attn_dot_rhs: x / f rows (16 bytes fp32, 8 bytes bf16) and the workspace "
                "must be aligned");
  if (flags & GNPDE_ADD_SOURCE)
    GNPDE_REQUIRE(ldx0 % 4 == 0 && rows_ok(x0), GNPDE_EUNSUPPORTED, "attn_dot_rhs: x0 rows must be aligned");
  if (stage) {
    bool ok = !stage->f_out || rows_ok(stage->f_out);
    for (int i = 0; i < stage->n_out; ++i) {
      ok = ok && rows_ok(stage->o[i].out) && (!stage->o[i].base || rows_ok(stage->o[i].base));
    }
    for (int j = 0; j < stage->nk; ++j) ok = ok && rows_ok(stage->k[j]);
    GNPDE_REQUIRE(ok && (!stage->dot_rows || aligned16(stage->dot_with)), GNPDE_EUNSUPPORTED,
                  "attn_dot_rhs: stage rows must be 16-byte aligned");
  }
  if (n_items == 0) return GNPDE_OK;
  DotArgs da;
  da.q = q;
  da.k = k;
  da.ldqk = ldqk;
  da.scale = kLog2e / sqrtf((float)dk);
  da.scale64 = 1.4426950408889634 / sqrt((double)dk);
  const int4* it = reinterpret_cast<const int4*>(items);
  int4* hv = reinterpret_cast<int4*>(heavy);
  const int lanes = (int)(C / 4);
  const int NA = (int)(heads * dk / 4), H = (int)heads;
  hipStream_t s = as_stream(stream);
  if (lanes <= 16)
    return launch_dot<16, T>(NA, H, it, n_items, hv, n_heavy, col, da, dst_stats, (int)C, ep, workspace, s);
  if (lanes <= 32)
    return launch_dot<32, T>(NA, H, it, n_items, hv, n_heavy, col, da, dst_stats, (int)C, ep, workspace, s);
  return launch_dot<64, T>(NA, H, it, n_items, hv, n_heavy, col, da, dst_stats, (int)C, ep, workspace, s);
}

extern "C" {

int gnpde_attn_dot_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                           const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads, int64_t dk,
                           const float* dst_stats, int64_t C, const float* x, int64_t ldx, const float* x0,
                           int64_t ldx0, const float* alpha, const float* beta, int flags, float* f, int64_t ldf,
                           float* workspace, int64_t n_slots, const gnpde_stage_epilogue_t* stage, void* stream) {
  return attn_dot_rhs_impl<float>(items, n_items, heavy, n_heavy, col, q, k, ldqk, heads, dk, dst_stats, C, x, ldx,
                                  x0, ldx0, alpha, beta, flags, f, ldf, workspace, n_slots, stage, stream);
}

int gnpde_attn_dot_rhs_bf16(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                            const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads,
                            int64_t dk, const float* dst_stats, int64_t C, const void* x, int64_t ldx, const void* x0,
                            int64_t ldx0, const float* alpha, const float* beta, int flags, void* f, int64_t ldf,
                            float* workspace, int64_t n_slots, const gnpde_stage_epilogue_t* stage, void* stream) {
  return attn_dot_rhs_impl<bf16>(items, n_items, heavy, n_heavy, col, q, k, ldqk, heads, dk, dst_stats, C,
                                 static_cast<const float*>(x), ldx, static_cast<const float*>(x0), ldx0, alpha, beta,
                                 flags, static_cast<float*>(f), ldf, workspace, n_slots, stage, stream);
}


}  // extern "C"
