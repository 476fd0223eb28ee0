// attention.hip — K2: edge-block segmented softmax of the attention RHS.
//
// One RHS of the transformer function needs, per edge e = (i -> j) and head h,
//   s_e,h   = score(q_i, k_j)                           (SDDMM)
//   a_e,h   = exp(s_e,h - max_g s) / (sum_g exp(. - max) + 1e-16)   over the group g
//             of e (its source i for attention_norm_idx 0, its destination j for 1)
//   w_e     = (1/H) sum_h a_e,h                          (head mean)
// and then ax_i = sum_e w_e x_j (K1, aggregate.hpp).  Reference:
//   SpGraphTransAttentionLayer.forward  src/function_transformer_attention.py:218-266
//   utils.softmax                       src/utils.py:116-127
//   multiply_attention head mean        src/function_transformer_attention.py:33-41
//
// Work decomposition (why not one group per wavefront): the graphs are
// power-law with a mean degree of ~7, so a wavefront per group leaves most
// lanes idle and serialises one dependent gather chain per few edges.  Here a
// wavefront takes an ITEM = a range of at most EB (<= 64) consecutive edges of
// the grouped CSR:
//   * a block of consecutive whole groups, packed greedily up to EB edges
//     (gnpde_seg_plan_build, once per graph), or
//   * a chunk of EB edges of a longer group (slot >= 0: partial statistics,
//     merged by the stats fixup of rhs.hip).
// Lane e of the wavefront owns edge e0 + e.  Scores are computed in the team
// layout (T = H*dk/4 lanes per edge, 16-byte q/k slices, up to kSegRounds
// rounds of 64/T edges, kSegBatch rounds of rows in flight together), moved to
// lane layout one head at a time, and the per-group max and sum-exp come from
// segmented inclusive scans over the lanes built from DPP row shifts and row
// broadcasts (VALU only, fixed order: deterministic), read back at the
// group's last lane.  (A design that also fused the x aggregation into this pass measured
// slower than this kernel + K1: the score latency in front of the gathers
// costs more than the 8 bytes per edge of weights)
//
// Outputs (OUT): kSegWeights = head-mean weights w[p] in grouped-CSR order
// (norm_idx 0, where the grouped CSR IS the aggregation CSR), chunk items ->
// partials; kSegStats = group statistics m[g,h] (fp64 max), rl[g,h] =
// 1/(sum + 1e-16) (norm_idx 1 over the CSC, read by the edge-parallel weight
// kernels of rhs.hip), chunk items -> partials; kSegChunkWeights = weights of
// the chunk items from the merged statistics of their group.
#include <type_traits>

#include "aggregate.hpp"
#include "rhs_host.hpp"

namespace gnpde {

constexpr int kSegRounds = 8;       // team rounds per item: EB = min(64, 8 * 64/T) edges
constexpr int kSegBatch = 4;        // rounds whose q/k slices are in flight together

enum { kSegWeights = 0, kSegStats = 1, kSegChunkWeights = 2 };

// ------------------------------------------------------------------ DPP cross-lane steps
// gfx9 DPP controls: row_shr:n (from lane - n inside a 16-lane row), row_bcast:15
// (lane 15 of each row to the next row), row_bcast:31 (lane 31 to rows 2-3).
// Lanes without a source keep `old`.  VALU only: no LDS-pipe permutes.
constexpr int kDppRowShr = 0x110;
constexpr int kDppBcast15 = 0x142;
constexpr int kDppBcast31 = 0x143;
constexpr int kDppQuadXor1 = 0xB1;  // quad_perm [1,0,3,2]
constexpr int kDppQuadXor2 = 0x4E;  // quad_perm [2,3,0,1]

template <int CTRL, int ROWS>
__device__ __forceinline__ int dpp_i(int old, int v) {
  return __builtin_amdgcn_update_dpp(old, v, CTRL, ROWS, 0xf, false);
}
template <int CTRL, int ROWS>
__device__ __forceinline__ float dpp_f(float old, float v) {
  return __builtin_bit_cast(float, dpp_i<CTRL, ROWS>(__builtin_bit_cast(int, old), __builtin_bit_cast(int, v)));
}
template <int CTRL, int ROWS>
__device__ __forceinline__ double dpp_d(double old, double v) {
  const long long o = __builtin_bit_cast(long long, old), x = __builtin_bit_cast(long long, v);
  const int lo = dpp_i<CTRL, ROWS>((int)o, (int)x);
  const int hi = dpp_i<CTRL, ROWS>((int)(o >> 32), (int)(x >> 32));
  return __builtin_bit_cast(double, ((long long)hi << 32) | (unsigned)lo);
}
template <int CTRL, int ROWS, class V>
__device__ __forceinline__ V dpp(V old, V v) {
  if constexpr (sizeof(V) == 8) return dpp_d<CTRL, ROWS>(old, v);
  else return dpp_f<CTRL, ROWS>(old, v);
}

// The six steps of a wave-wide inclusive scan: row_shr 1,2,4,8, then
// row_bcast15 into rows 1 and 3, then row_bcast31 into rows 2 and 3.
// seg_flags: bit k set when the source lane of step k is in the same group.
__device__ __forceinline__ unsigned seg_flags(int grp) {
  unsigned f = 0;
  f |= (dpp_i<kDppRowShr + 1, 0xf>(-1, grp) == grp) ? 1u : 0u;
  f |= (dpp_i<kDppRowShr + 2, 0xf>(-1, grp) == grp) ? 2u : 0u;
  f |= (dpp_i<kDppRowShr + 4, 0xf>(-1, grp) == grp) ? 4u : 0u;
  f |= (dpp_i<kDppRowShr + 8, 0xf>(-1, grp) == grp) ? 8u : 0u;
  f |= (dpp_i<kDppBcast15, 0xa>(-1, grp) == grp) ? 16u : 0u;
  f |= (dpp_i<kDppBcast31, 0xc>(-1, grp) == grp) ? 32u : 0u;
  return f;
}

template <bool MAX, class V>
__device__ __forceinline__ V seg_scan(V v, unsigned f) {
  const V id = MAX ? (V)-INFINITY : (V)0;
  auto op = [](V a, V b) { return MAX ? (a > b ? a : b) : a + b; };
  V u;
  u = dpp<kDppRowShr + 1, 0xf>(id, v);
  if (f & 1u) v = op(v, u);
  u = dpp<kDppRowShr + 2, 0xf>(id, v);
  if (f & 2u) v = op(v, u);
  u = dpp<kDppRowShr + 4, 0xf>(id, v);
  if (f & 4u) v = op(v, u);
  u = dpp<kDppRowShr + 8, 0xf>(id, v);
  if (f & 8u) v = op(v, u);
  u = dpp<kDppBcast15, 0xa>(id, v);
  if (f & 16u) v = op(v, u);
  u = dpp<kDppBcast31, 0xc>(id, v);
  if (f & 32u) v = op(v, u);
  return v;
}

// sum over the S lanes of a head segment: DPP quad permutes for the first two
// steps, LDS permutes beyond (S <= 16)
__device__ __forceinline__ float head_sum(float v, int S) {
  if (S >= 2) v += dpp_f<kDppQuadXor1, 0xf>(0.f, v);
  if (S >= 4) v += dpp_f<kDppQuadXor2, 0xf>(0.f, v);
  for (int o = 4; o < S; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// team_score_regs with the DPP head reduction (scaled_dot; other modes as in scores.hpp)
__device__ __forceinline__ float seg_team_score(const ScoreArgs& sa, const float (&q)[4], const float (&k)[4], int S) {
  if (sa.mode == GNPDE_SCORE_DOT) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) a = fmaf(q[i], k[i], a);
    return head_sum(a, S) * rsqrtf((float)sa.dk);
  }
  return team_score_regs<4>(sa, q, k, S);
}

// ------------------------------------------------------------------ long groups (reference statistics)
// Reference-score statistics of destination groups longer than a wavefront's
// 64-edge block (ref_stats_kernel), one wavefront per item, lanes striding
// (kSegLongU edges per lane, one pass of up to kSegLongMax edges), each lane an
// online (max, sum-exp) per head, then a fixed xor tree across the lanes:
//   * LONG items (slot field -2): a whole group of at most kSegLongMax edges;
//   * HUB CHUNK items {e_begin, e_end, slot, hub}: kSegLongMax-edge chunks of a
//     longer group.  The chunk's (M, L) per head goes write-through to its
//     partial slot; the chunk wave then takes an arrival ticket on the hub table
//     entry heavy[hub] = {group, first_slot, n_chunks, ticket}, and the last to
//     arrive merges the slots (stats_merge_store: lanes over chunks, fixed xor
//     tree, so the result does not depend on the arrival order) and resets the
//     ticket.  Round 3 ran each hub group as one 1024-thread workgroup (mostly
//     idle lanes, 16 wave slots held per group): the kernel took 20.9 us on
//     G-arxiv's CSC, bound by those groups.
// timing probes of experiment builds (GNPDE_RS_SKIP, launch_ref_stats): 1 / 2 skip the
// hub + long / the short items, 4 stops a long item after its passes, 5 after its item load
#if GNPDE_EXPERIMENTS
__constant__ int g_rs_skip = 0;
__device__ __forceinline__ int rs_skip() { return g_rs_skip; }
#else
__device__ __forceinline__ int rs_skip() { return 0; }
#endif

constexpr int kSegLongU = 8;                   // edges per lane
constexpr int kSegLongMax = kWave * kSegLongU;  // 512: one pass

// node scores cs[src[u], 0..MAXH) of U sources (src < 0: row 0, unused): two
// heads as one 16-byte load — one gather instruction instead of two (random
// 8-byte gathers are bound by the address unit, one cache line per lane): G-arxiv
// CSC statistics 21.0 -> 19.3 us, hub groups alone 15.2 -> 13.7 us.  (Two-phase
// max-then-sum reductions instead of merging online pairs: hub / long groups 10.6 /
// 6.9 us, but the scores kept in registers between the phases cost the short
// items their occupancy, 22.7 us in all; reloading them, 20.2 us.)
template <int U, int MAXH>
__device__ __forceinline__ void load_cs_rows(const ScoreArgs& sa, const int (&src)[U], double (&v)[U][MAXH]) {
  const int H = sa.H;
  if constexpr (MAXH == 2) {  // launch_ref_stats: MAXH == 2 means H == 2 and 16-byte aligned rows
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const double2 t = *reinterpret_cast<const double2*>(sa.cs + (int64_t)max(src[u], 0) * 2);
      v[u][0] = t.x;
      v[u][1] = t.y;
    }
  } else {
#pragma unroll
    for (int u = 0; u < U; ++u)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) v[u][h] = h < H ? sa.cs[(int64_t)max(src[u], 0) * H + h] : 0.0;
  }
}

template <int U, int MAXH>
__device__ __forceinline__ void push_edges(int pb, int stride, int e1, const int* __restrict__ gidx,
                                           const ScoreArgs& sa, double (&M)[MAXH], float (&L)[MAXH]) {
  const int H = sa.H;
  int src[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int p = pb + stride * u;
    src[u] = p < e1 ? gidx[p] : -1;
  }
  double v[U][MAXH];
  load_cs_rows<U, MAXH>(sa, src, v);
#pragma unroll
  for (int u = 0; u < U; ++u)
#pragma unroll
    for (int h = 0; h < MAXH; ++h)
      if (src[u] >= 0 && h < H) online_push(M[h], L[h], v[u][h]);
}

template <int MAXH>
__device__ __forceinline__ void wave_merge(double (&M)[MAXH], float (&L)[MAXH]) {
  lanes_merge<MAXH>(M, L);
}

// at most kSegLongMax edges [e0, e1) by one wavefront: (M, L) per head, every lane
template <int MAXH>
__device__ __forceinline__ void long_item_stats(int e0, int e1, const int* __restrict__ gidx, const ScoreArgs& sa,
                                                double (&M)[MAXH], float (&L)[MAXH]) {
  const int lane = threadIdx.x & 63;
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
  }
  // one pass of kSegLongU edges per lane (more heads: passes of fewer, for registers)
  constexpr int LU = MAXH <= 2 ? kSegLongU : 2;
#pragma unroll(MAXH <= 2 ? kSegLongU / LU : 1)
  for (int ps = 0; ps < kSegLongU / LU; ++ps) {
    if (e0 + ps * LU * kWave >= e1) break;  // wave-uniform: an item of fewer edges skips the empty passes
    push_edges<LU, MAXH>(e0 + lane + ps * LU * kWave, kWave, e1, gidx, sa, M, L);
  }
  if (GNPDE_EXPERIMENTS && rs_skip() == 4) return;
  wave_merge<MAXH>(M, L);
}

// a hub chunk: partials write-through, arrival ticket, the last arrival merges
template <int MAXH>
__device__ __forceinline__ void hub_chunk_stats(int e0, int e1, int slot, int hub, const int* __restrict__ gidx,
                                                const ScoreArgs& sa, int4* heavy, double* __restrict__ partials,
                                                double* m, float* rl, float* mr) {
  const int lane = threadIdx.x & 63;
  const int H = sa.H;
  double M[MAXH];
  float L[MAXH];
  long_item_stats<MAXH>(e0, e1, gidx, sa, M, L);
  const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
  const int64_t pb = (int64_t)slot * 2 * H;
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    const bool st = lane == 0 && h < H;
    buf_store_wt_f64(rp, st ? (uint32_t)((pb + h) * 8) : kBufNone, M[h]);
    buf_store_wt_f64(rp, st ? (uint32_t)((pb + H + h) * 8) : kBufNone, (double)L[h]);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  int ticket = 0;
  if (lane == 0) ticket = __hip_atomic_fetch_add(&heavy[hub].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
  ticket = __shfl(ticket, 0);
  const int4 hv = heavy[hub];
  if (ticket != uniform(hv.z) - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  stats_merge_store_heads<MAXH>(uniform(hv.x), uniform(hv.y), uniform(hv.z), H, partials, m, rl, mr);
  if (lane == 0) __hip_atomic_store(&heavy[hub].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <bool REF, int OUT>
__global__ __launch_bounds__(256) void seg_softmax_kernel(const int4* __restrict__ items, int n_items,
                                                           const int* __restrict__ rowptr,
                                                           const int* __restrict__ rowidx,
                                                           const int* __restrict__ gidx, int group_is_dst,
                                                           ScoreArgs sa, Team tm, float* __restrict__ w,
                                                           double* __restrict__ m, float* __restrict__ rl,
                                                           float* __restrict__ mr, double* __restrict__ partials,
                                                           int4* heavy, int n_heavy) {
  using S_t = typename std::conditional<REF, double, float>::type;
  const int lane = threadIdx.x & 63;
  const int item = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (item >= n_items) return;
  const int4 it = items[item];
  const int e0 = uniform(it.x), e1 = uniform(it.y), slot = uniform(it.z);
  const int n = e1 - e0;
  if (n <= 0) return;
  const bool live = lane < n;
  const int p = e0 + min(lane, n - 1);
  const int grp = rowidx[p];
  const int oth = gidx[p];
  const int src = group_is_dst ? oth : grp;
  const int dst = group_is_dst ? grp : oth;
  const int seg_end = min(rowptr[grp + 1], e1) - 1 - e0;  // last lane of this lane's group inside the item
  const unsigned same = seg_flags(grp) & (live ? 0x3fu : 0u);  // all lanes run the DPP steps

  // team-layout scores (per-edge modes): lane (team, t) holds the score of edge
  // r*ER + team for head t/S; the q and k slices of kSegBatch rounds are in flight together
  const int T = REF ? 1 : tm.T, S = REF ? 1 : tm.S, ER = kWave / T;
  const int team = lane / T, t = lane % T;
  float sc[REF ? 1 : kSegRounds];
  if constexpr (!REF) {
#pragma unroll
    for (int b = 0; b < kSegRounds; b += kSegBatch) {
      if (b * ER < n) {
        float qv[kSegBatch][4], kv[kSegBatch][4];
#pragma unroll
        for (int r = 0; r < kSegBatch; ++r) {
          if ((b + r) * ER < n) {
            const int sl = min((b + r) * ER + team, n - 1);
            team_row<4>(sa, sa.q, __shfl(src, sl), t, qv[r]);
            team_row<4>(sa, sa.k, __shfl(dst, sl), t, kv[r]);
          }
        }
#pragma unroll
        for (int r = 0; r < kSegBatch; ++r)
          if ((b + r) * ER < n) sc[b + r] = seg_team_score(sa, qv[r], kv[r], S);  // full-wave cross-lane ops
      }
    }
  }
  const int round_of_lane = lane / ER, team_src = (lane % ER) * T;

  const int H = sa.H;
  // (Gathering every head's cs[src] before the head loop measured slower:
  // 16.5 against 15.3 us for the G-arxiv CSC statistics.)
  float wsum = 0.f;
  for (int h = 0; h < H; ++h) {
    S_t v;
    if constexpr (REF) {
      v = live ? sa.cs[(int64_t)src * H + h] : -INFINITY;
    } else {
      v = -INFINITY;
#pragma unroll
      for (int r = 0; r < kSegRounds; ++r) {
        if (r * ER < n) {
          const float x = __shfl(sc[r], team_src + h * S);
          if (round_of_lane == r) v = x;
        }
      }
      if (!live) v = -INFINITY;
    }
    if constexpr (OUT == kSegChunkWeights) {
      const int64_t gi = (int64_t)grp * H + h;
      wsum += live ? expf((float)((double)v - m[gi])) * rl[gi] : 0.f;
    } else {
      const S_t M = __shfl(seg_scan<true>(v, same), seg_end);
      const float e = live ? expf((float)(v - M)) : 0.f;
      const float Ls = __shfl(seg_scan<false>(e, same), seg_end);
      if (slot >= 0) {  // chunk of a long group: one segment, partial statistics
        if (lane == 0) {
          partials[(int64_t)slot * 2 * H + h] = (double)M;
          partials[(int64_t)slot * 2 * H + H + h] = (double)Ls;
        }
      } else if constexpr (OUT == kSegWeights) {
        wsum += e / (Ls + kSoftmaxEps);
      } else {
        if (live && lane == seg_end) store_stats(m, rl, mr, grp, H, h, (double)M, Ls);
      }
    }
  }
  if constexpr (OUT == kSegWeights || OUT == kSegChunkWeights) {
    if (live && (OUT == kSegChunkWeights || slot < 0)) w[p] = wsum / (float)H;
  }
}

// ------------------------------------------------------------------ reference statistics
// The reference scores' destination statistics (norm_idx 1) in one launch of
// 1024-thread workgroups over a plan of HUB items (one workgroup each), then
// LONG items (one wavefront each), then SHORT items (whole groups packed up to 64
// edges, NI per wavefront with every load of all NI items issued before any
// arithmetic: item -> {group id, source id} -> the sources' node scores is a
// chain of three dependent loads, so two items per wave overlap their chains).
// A lane's segment end comes from a ballot of group changes (no rowptr gather).
// Same arithmetic as seg_softmax_kernel<true, kSegStats>: segmented max,
// exp(v - M), segmented sum, in the same lane order.
#ifndef GNPDE_RS_NI
#define GNPDE_RS_NI 1
#endif
// short items per wavefront: round 3 (1024-thread workgroups) 1 / 2 / 4 = 20.9 / 21.0 / 23.1 us;
// round 4 (256-thread workgroups, hub chunks) 16.25 / 16.9 / 19.1 us (tools/ab_stats.sh)
constexpr int kRefStatsNI = GNPDE_RS_NI;

template <int NI, int MAXH>
__global__ __launch_bounds__(256) void ref_stats_kernel(const int4* __restrict__ items, int n_items, int n_hub,
                                                         int n_long, const int* __restrict__ rowidx,
                                                         const int* __restrict__ gidx, ScoreArgs sa, int4* heavy,
                                                         double* __restrict__ partials, double* __restrict__ m,
                                                         float* __restrict__ rl, float* __restrict__ mr) {
  const int lane = threadIdx.x & 63;
  const int wid = uniform((int)blockIdx.x * kWavesPerBlock + (int)(threadIdx.x >> 6));
  if constexpr (GNPDE_EXPERIMENTS) {  // timing probes: 1 skips the hub / long items, 2 the short ones
    if (rs_skip() == 1 && wid < n_hub + n_long) return;
    if (rs_skip() == 2 && wid >= n_hub + n_long) return;
  }
  if (wid < n_hub + n_long) {
    const int4 it = items[wid];
    if (GNPDE_EXPERIMENTS && rs_skip() == 5 && it.x == -7) return;  // (never: keeps the item load)
    if (GNPDE_EXPERIMENTS && rs_skip() == 5) {
      if (lane == 0 && it.y < 0) m[0] = 0.0;  // a use of the load, never taken
      return;
    }
    if (wid < n_hub) {
      hub_chunk_stats<MAXH>(uniform(it.x), uniform(it.y), uniform(it.z), uniform(it.w), gidx, sa, heavy, partials, m,
                            rl, mr);
      return;
    }
    double M[MAXH];
    float L[MAXH];
    long_item_stats<MAXH>(uniform(it.x), uniform(it.y), gidx, sa, M, L);
    if (lane == 0)
#pragma unroll
      for (int h = 0; h < MAXH; ++h)
        if (h < sa.H) store_stats(m, rl, mr, uniform(it.w), sa.H, h, M[h], L[h]);
    return;
  }
  const int base = n_hub + n_long + (wid - n_hub - n_long) * NI;
  if (base >= n_items) return;
  const int H = sa.H;
  int e0[NI], n[NI], grp[NI], src[NI];
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int4 it = base + i < n_items ? items[base + i] : make_int4(0, 0, -1, 0);
    e0[i] = uniform(it.x);
    n[i] = uniform(it.y) - e0[i];
  }
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    const int p = e0[i] + min(lane, max(n[i] - 1, 0));
    grp[i] = n[i] > 0 ? rowidx[p] : 0;
    src[i] = n[i] > 0 ? gidx[p] : 0;
  }
  double v[NI][MAXH];
  load_cs_rows<NI, MAXH>(sa, src, v);
#pragma unroll
  for (int i = 0; i < NI; ++i) {
    if (n[i] > 0) {  // wave-uniform
      const bool live = lane < n[i];
      const int nxt = __shfl(grp[i], min(lane + 1, 63));
      const unsigned long long ends = __ballot(live && (lane == n[i] - 1 || nxt != grp[i]));
      const int seg_end = lane + (int)__builtin_ctzll(ends >> lane | (1ull << 63 >> lane));
      const unsigned same = seg_flags(grp[i]) & (live ? 0x3fu : 0u);
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        if (h < H) {
          const double x = live ? v[i][h] : -INFINITY;
          const double M = __shfl(seg_scan<true>(x, same), seg_end);
          const float e = live ? expf((float)(x - M)) : 0.f;
          const float Ls = __shfl(seg_scan<false>(e, same), seg_end);
          if (live && lane == seg_end) store_stats(m, rl, mr, grp[i], H, h, M, Ls);
        }
      }
    }
  }
}

template <int NI>
static int launch_ref_stats(const int4* items, int64_t n_items, int64_t n_hub, int64_t n_long, const int* rowidx,
                            const int* gidx, const ScoreArgs& sa, int4* heavy, double* partials, double* m, float* rl,
                            float* mr, hipStream_t s) {
#if GNPDE_EXPERIMENTS
  static const bool once = [] {  // GNPDE_RS_SKIP: the kernel's timing probes (before any capture)
    const char* e = std::getenv("GNPDE_RS_SKIP");
    const int v = e ? std::atoi(e) : 0;
    return hipMemcpyToSymbol(HIP_SYMBOL(g_rs_skip), &v, sizeof(int)) == hipSuccess;
  }();
  (void)once;
#endif
  const int64_t waves = n_hub + n_long + ceil_div(n_items - n_hub - n_long, (int64_t)NI);
  const unsigned grid = (unsigned)ceil_div(waves, (int64_t)kWavesPerBlock);
#define GNPDE_RS(M)                                                                                            \
  ref_stats_kernel<NI, M><<<grid, kBlock, 0, s>>>(items, (int)n_items, (int)n_hub, (int)n_long, rowidx, gidx, sa, \
                                                   heavy, partials, m, rl, mr)
  if (sa.H <= 1)
    GNPDE_RS(1);
  else if (sa.H <= 2 && aligned16(sa.cs))  // MAXH 2: two heads, 16-byte node-score rows
    GNPDE_RS(2);
  else if (sa.H <= 4)
    GNPDE_RS(4);
  else if (sa.H <= 8)
    GNPDE_RS(8);
  else
    GNPDE_RS(16);
#undef GNPDE_RS
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

template <bool REF, int OUT>
static int launch_seg(const int4* items, int64_t n, const int* rowptr, const int* rowidx, const int* gidx, int gid,
                      const ScoreArgs& sa, const Team& tm, float* w, double* m, float* rl, float* mr,
                      double* partials, int4* heavy, int n_heavy, hipStream_t s) {
  if (n <= 0) return GNPDE_OK;
  seg_softmax_kernel<REF, OUT><<<(unsigned)ceil_div(n, kWavesPerBlock), kBlock, 0, s>>>(
      items, (int)n, rowptr, rowidx, gidx, gid, sa, tm, w, m, rl, mr, partials, heavy, n_heavy);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_seg_long_edges(void) { return kSegLongMax; }

// edges one pass of a long statistics item covers (long_item_stats: kSegLongU edges
// per lane up to two heads, 2 per lane beyond): the plan's long-item size when every
// wavefront should finish in one pass (latency-bound small graphs)
int gnpde_seg_long_pass_edges(int64_t heads) { return kWave * (heads <= 2 ? kSegLongU : 2); }

int gnpde_seg_block_edges(int mode, int64_t heads, int64_t dk) {
  if (mode == GNPDE_SCORE_REFERENCE || mode == GNPDE_SCORE_UNIFORM) return kWave;
  if (heads < 1 || dk < 4 || dk % 4 != 0) return 0;
  const int64_t S = dk / 4, T = heads * S;
  if ((S & (S - 1)) || (T & (T - 1)) || T > kWave) return 0;
  return (int)std::min<int64_t>(kWave, kSegRounds * (kWave / T));
}

int gnpde_seg_plan_build(const int32_t* rowptr, int64_t R, int32_t eb, int32_t* items, int64_t items_capacity,
                         int32_t* chunk_items, int64_t chunks_capacity, int32_t* heavy, int64_t heavy_capacity,
                         int64_t* n_items, int64_t* n_chunks, int64_t* n_heavy) {
  GNPDE_REQUIRE(rowptr && items && chunk_items && heavy && n_items && n_chunks && n_heavy, GNPDE_EINVAL,
                "seg_plan_build: NULL pointer");
  GNPDE_REQUIRE(R >= 0 && eb >= 1 && eb <= kWave, GNPDE_EINVAL, "seg_plan_build: bad R / eb");
  int64_t ni = 0, nc = 0, nh = 0;
  int64_t b0 = -1, b1 = -1, bg = -1;  // the open block [b0, b1), first group bg
  auto close = [&]() -> bool {
    if (b0 < 0) return true;
    if (ni >= items_capacity) return false;
    int32_t* o = items + 4 * ni++;
    o[0] = (int32_t)b0; o[1] = (int32_t)b1; o[2] = -1; o[3] = (int32_t)bg;
    b0 = -1;
    return true;
  };
  for (int64_t r = 0; r < R; ++r) {
    const int64_t s0 = rowptr[r], s1 = rowptr[r + 1], d = s1 - s0;
    GNPDE_REQUIRE(d >= 0, GNPDE_EINVAL, "seg_plan_build: rowptr not monotone at %lld", (long long)r);
    if (d == 0) continue;  // empty groups: no edges, nothing to compute
    if (d > eb) {          // long group: eb-edge chunks with partial statistics
      GNPDE_REQUIRE(close(), GNPDE_EINVAL, "seg_plan_build: items capacity");
      const int64_t nch = (d + eb - 1) / eb;
      GNPDE_REQUIRE(nc + nch <= chunks_capacity && nh < heavy_capacity, GNPDE_EINVAL, "seg_plan_build: chunk capacity");
      int32_t* hv = heavy + 4 * nh++;
      hv[0] = (int32_t)r; hv[1] = (int32_t)nc; hv[2] = (int32_t)nch; hv[3] = 0;
      for (int64_t c = 0; c < nch; ++c) {
        int32_t* o = chunk_items + 4 * nc;
        o[0] = (int32_t)(s0 + c * eb); o[1] = (int32_t)std::min(s1, s0 + (c + 1) * eb); o[2] = (int32_t)nc;
        o[3] = (int32_t)r;
        ++nc;
      }
      continue;
    }
    if (b0 >= 0 && s1 - b0 <= eb) {  // non-empty groups are contiguous in edge order
      b1 = s1;
      continue;
    }
    GNPDE_REQUIRE(close(), GNPDE_EINVAL, "seg_plan_build: items capacity");
    b0 = s0;
    b1 = s1;
    bg = r;
  }
  GNPDE_REQUIRE(close(), GNPDE_EINVAL, "seg_plan_build: items capacity");
  *n_items = ni;
  *n_chunks = nc;
  *n_heavy = nh;
  return GNPDE_OK;
}

int gnpde_seg_softmax_f32(const int32_t* items, int64_t n_items, int64_t n_hub_items, int64_t n_long_items,
                          const int32_t* chunk_items,
                          int64_t n_chunk_items, int32_t* heavy, int64_t n_heavy, const int32_t* rowptr,
                          const int32_t* rowidx,
                          const int32_t* gidx, int group_is_dst, int out_kind, int mode, int64_t heads, int64_t dk,
                          const double* cs, const float* q, const float* k, int64_t ldqk, float score_p0,
                          float score_p1, float* w, double* m, float* rl, float* mr, double* partials,
                          void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE(out_kind == 0 || out_kind == 1, GNPDE_EINVAL, "seg_softmax: out_kind must be 0 (weights) or 1 (stats)");
  GNPDE_REQUIRE(mode != GNPDE_SCORE_UNIFORM, GNPDE_EUNSUPPORTED, "seg_softmax: uniform scores need no softmax pass");
  GNPDE_REQUIRE(!(mode == GNPDE_SCORE_REFERENCE && out_kind == 0), GNPDE_EUNSUPPORTED,
                "seg_softmax: reference scores grouped by source are uniform");
  GNPDE_REQUIRE(n_items >= 0 && n_chunk_items >= 0 && n_heavy >= 0 && n_items + n_chunk_items < INT32_MAX &&
                    n_hub_items >= 0 && n_long_items >= 0 && n_hub_items + n_long_items <= n_items,
                GNPDE_EINVAL, "seg_softmax: bad item counts");
  GNPDE_REQUIRE(n_hub_items + n_long_items == 0 || (mode == GNPDE_SCORE_REFERENCE && out_kind == 1 && group_is_dst &&
                                                    n_chunk_items == 0),
                GNPDE_EINVAL, "seg_softmax: hub / long items are for the reference statistics (norm_idx 1) only");
  GNPDE_REQUIRE(gnpde_seg_block_edges(mode, heads, dk) > 0, GNPDE_EUNSUPPORTED,
                "seg_softmax: per-edge scores need dk %% 4 == 0 and power-of-two dk/4, heads*dk/4 <= 64");
  if (n_items + n_chunk_items == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowptr && rowidx && gidx, GNPDE_EINVAL, "seg_softmax: NULL graph arrays");
  GNPDE_REQUIRE(n_items == 0 || items, GNPDE_EINVAL, "seg_softmax: NULL items");
  GNPDE_REQUIRE(n_chunk_items == 0 || (chunk_items && heavy && n_heavy > 0 && partials &&
                                      ((m && rl) || (out_kind == 1 && mr))),
                GNPDE_EINVAL, "seg_softmax: chunk items need heavy, partials and m/rl scratch");
  if (out_kind == 0) GNPDE_REQUIRE(w != nullptr, GNPDE_EINVAL, "seg_softmax: NULL w");
  if (out_kind == 1) GNPDE_REQUIRE((m && rl) || mr, GNPDE_EINVAL, "seg_softmax: no output (m/rl or the packed records)");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  Team tm{1, 1};
  if (mode != GNPDE_SCORE_REFERENCE) {
    tm = team_geometry(sa);
    GNPDE_REQUIRE(tm.T > 0, GNPDE_EUNSUPPORTED, "seg_softmax: q/k must be 16-byte aligned with ldqk %% 4 == 0");
  }
  hipStream_t s = as_stream(stream);
  const int4* it = reinterpret_cast<const int4*>(items);
  const int4* ch = reinterpret_cast<const int4*>(chunk_items);
  int4* hv = reinterpret_cast<int4*>(heavy);
  const bool ref = mode == GNPDE_SCORE_REFERENCE;
  GNPDE_REQUIRE((uint64_t)(n_items + n_chunk_items) * 2 * heads * 8 < kBufRecords && n_heavy < INT32_MAX,
                GNPDE_EUNSUPPORTED, "seg_softmax: partials too large");
#define GNPDE_SEG(R, O, ITEMS, N)                                                                                  \
  launch_seg<R, O>(ITEMS, N, rowptr, rowidx, gidx, group_is_dst, sa, tm, w, m, rl, (O) == kSegStats ? mr : nullptr, \
                   partials, hv, (int)n_heavy, s)
  // whole-group items and long-group chunks share one kernel (the slot field
  // tells them apart): one launch when the caller stores them back to back
  const bool adjacent = n_items > 0 && n_chunk_items > 0 && ch == it + n_items;
  const int64_t n_first = adjacent ? n_items + n_chunk_items : n_items;
  const int64_t n_second = adjacent ? 0 : n_chunk_items;
  if (ref && out_kind == 1 && n_chunk_items == 0 && group_is_dst) {
    // the reference statistics of the attention RHS: hub chunks, long groups, then short items
    GNPDE_REQUIRE((uint64_t)n_items < (uint64_t)INT32_MAX / kWavesPerBlock, GNPDE_EUNSUPPORTED,
                  "seg_softmax: too many items");
    GNPDE_REQUIRE(n_hub_items == 0 || (heavy && n_heavy > 0 && partials), GNPDE_EINVAL,
                  "seg_softmax: hub chunk items need the hub table (heavy) and partials");
    return launch_ref_stats<kRefStatsNI>(it, n_items, n_hub_items, n_long_items, rowidx, gidx, sa, hv, partials, m, rl,
                                          mr, s);
  }
  if (out_kind == 0) {
    rc = GNPDE_SEG(false, kSegWeights, it, n_first);
    if (!rc) rc = GNPDE_SEG(false, kSegWeights, ch, n_second);
  } else if (ref) {
    rc = GNPDE_SEG(true, kSegStats, it, n_first);
    if (!rc) rc = GNPDE_SEG(true, kSegStats, ch, n_second);
  } else {
    rc = GNPDE_SEG(false, kSegStats, it, n_first);
    if (!rc) rc = GNPDE_SEG(false, kSegStats, ch, n_second);
  }
  if (rc || n_chunk_items == 0) return rc;
  rc = launch_stats_fixup(hv, n_heavy, (int)heads, partials, m, rl, out_kind == 1 ? mr : nullptr, s);
  if (rc || out_kind == 1) return rc;
  return GNPDE_SEG(false, kSegChunkWeights, ch, n_chunk_items);
#undef GNPDE_SEG
}

}  // extern "C"
