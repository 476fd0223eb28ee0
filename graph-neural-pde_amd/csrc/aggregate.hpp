// aggregate.hpp — the gather-aggregate engine shared by the Laplacian RHS (K1)
// and the attention RHS (K3): one wavefront per work item (a whole CSR row or a
// chunk of a hub row), rows of x gathered with 16-byte loads, the RHS epilogue
// fused.  Hub rows are split into chunk items whose partial sums are combined
// inside the same launch by the chunk that finishes last (arrival ticket on the
// hub's plan entry; fixed summation order, so deterministic; no float atomics).
#pragma once
#include <algorithm>
#include <type_traits>

#include "common.hpp"

namespace gnpde {

// ------------------------------------------------------------------ weight policies
// A policy splits the weight of CSR position p (row, destination c) into
// load() — the raw operands, issued with the column index — and finish() —
// the arithmetic, run once the first gathers of x are in flight, so the
// weight's memory latency overlaps the row gathers instead of preceding them.
//
// Plain per-edge weights (Laplacian RHS, function_laplacian_diffusion.py:54-57).
struct PlainWeights {
  const float* __restrict__ w;
  struct Raw {
    float w;
  };
  __device__ __forceinline__ Raw load(int /*row*/, int p, int /*c*/) const { return Raw{w[p]}; }
  __device__ __forceinline__ float finish(int /*row*/, const Raw& r) const { return r.w; }
};

// Reference-mode (fork scaled_dot) attention under destination-grouped softmax
// (attention_norm_idx 1), head-mean taken on the fly: the score of an edge is
// the node score cs[row, h] of its source (the aggregating row), the group
// statistics m, rl belong to its destination c.  Same arithmetic, in the same
// order, as attn_weights_kernel (rhs.hip), so fusing it into K1 changes no
// bit; it saves the separate weights pass and its [nnz] round trip.
// MAXH > 0: heads <= MAXH, the per-edge statistics are loaded up front;
// MAXH == 0: any heads <= 16, loaded in finish().  EXACT (heads == MAXH == 2,
// m 16-byte and rl 8-byte aligned): one 16-B load of m[c,:] and one 8-B load
// of rl[c,:] per edge instead of four scalar gathers.
// REC (with EXACT): m and rl come from the packed statistics records of the
// destinations (rec, stats_record_floats(2) = 4 floats: m[0..1], rl[0..1]):
// one 16-byte load per edge, a quarter of a cache line, instead of two lines of
// the separate arrays; the same values (the stored max is fp32-exact in both
// forms) and the same finish(), so the same bits.
template <int MAXH, bool EXACT = false, bool REC = false>
struct RefDstSoftmaxWeights {
  const double* __restrict__ cs;
  const double* __restrict__ m;
  const float* __restrict__ rl;
  int H;
  const float* __restrict__ rec;
  struct Raw {
    double mm[MAXH > 0 ? MAXH : 1];
    float rr[MAXH > 0 ? MAXH : 1];
    int c;
  };
  __device__ __forceinline__ Raw load(int /*row*/, int /*p*/, int c) const {
    Raw r;
    r.c = c;
    if constexpr (EXACT && REC) {
      static_assert(MAXH == 2 && stats_record_floats(2) == 4, "two-head records are 16 bytes");
      const float4 v = *reinterpret_cast<const float4*>(rec + (int64_t)c * 4);
      r.mm[0] = (double)v.x;
      r.mm[1] = (double)v.y;
      r.rr[0] = v.z;
      r.rr[1] = v.w;
    } else if constexpr (EXACT) {
      static_assert(MAXH == 2, "EXACT statistics loads are written for two heads");
      const double2 mv = *reinterpret_cast<const double2*>(m + (int64_t)c * 2);
      const float2 rv = *reinterpret_cast<const float2*>(rl + (int64_t)c * 2);
      r.mm[0] = mv.x;
      r.mm[1] = mv.y;
      r.rr[0] = rv.x;
      r.rr[1] = rv.y;
    } else if constexpr (MAXH > 0) {
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        const int hh = h < H ? h : 0;
        r.mm[h] = m[(int64_t)c * H + hh];
        r.rr[h] = rl[(int64_t)c * H + hh];
      }
    }
    return r;
  }
  __device__ __forceinline__ float finish(int row, const Raw& r) const {
    float acc = 0.f;
    if constexpr (MAXH > 0) {
#pragma unroll
      for (int h = 0; h < MAXH; ++h)
        if (h < H) acc += expf((float)(cs[(int64_t)row * H + h] - r.mm[h])) * r.rr[h];
    } else {
      for (int h = 0; h < H; ++h)
        acc += expf((float)(cs[(int64_t)row * H + h] - m[(int64_t)r.c * H + h])) * rl[(int64_t)r.c * H + h];
    }
    return acc / (float)H;
  }
};

template <class WP>
__host__ __device__ inline PlainWeights as_plain(const WP& wp) {
  if constexpr (std::is_same<WP, PlainWeights>::value) return wp;
  else return PlainWeights{nullptr};  // never launched (launch_agg_cfg)
}

// ------------------------------------------------------------------ hub rows
// Lane groups of the hub combine are powers of two (an xor tree joins them):
// a geometry with GL = 21 lanes per row (three bf16 rows of 168 columns per
// wavefront) combines its hub rows with 32-lane groups.
constexpr int pow2_ceil(int v) { return v <= 1 ? 1 : 2 * pow2_ceil((v + 1) / 2); }

// Sum the nch chunk partials of hub row `row` (slots first .. first+nch-1), then
// run the epilogue.  GL lanes cover the columns; the 64/GL lane groups take
// chunks g, g+G, ... and are combined by a fixed xor tree (deterministic).
template <int VEC, int GL, int STG, class T>
__device__ __forceinline__ void hub_combine(int row, int first, int nch, int C, const Epi& ep,
                                            const float* __restrict__ partials) {
  constexpr int G = kWave / GL;
  const int lane = threadIdx.x & 63;
  const int g = lane / GL, gl = lane % GL;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart[2] = {0.0, 0.0};
  for (int c0 = 0; c0 < C; c0 += GL * VEC) {
    const int cc = c0 + gl * VEC;
    const bool live = cc < C;
    float s[VEC];
#pragma unroll
    for (int t = 0; t < VEC; ++t) s[t] = 0.f;
#pragma unroll 4
    for (int c = g; c < nch; c += G) {
      float v[VEC];
      if (live) {
        load_vec<VEC>(partials + (int64_t)(first + c) * C + cc, v);
      } else {
#pragma unroll
        for (int t = 0; t < VEC; ++t) v[t] = 0.f;
      }
#pragma unroll
      for (int t = 0; t < VEC; ++t) s[t] += v[t];
    }
#pragma unroll
    for (int o = GL; o < kWave; o <<= 1)
#pragma unroll
      for (int t = 0; t < VEC; ++t) s[t] += __shfl_xor(s[t], o);
    if (g == 0 && live) epilogue_store<VEC, STG, T>(ep, row, cc, s, a, b, dpart);
  }
  epi_rowsums<GL, STG, T>(ep, row, dpart, 0, lane == 0);  // wave-uniform
}

// The sum of the nch chunk partials of a hub row (slots first .. first+nch-1),
// computed by all 64 lanes: lane groups of GLp = pow2_ceil(GL) lanes take chunks
// g, g+G, ... (4 loads in flight), joined by a fixed xor tree — the order of
// hub_combine, so the same bits.  Every lane ends with the sums of the columns
// (ch*GLp + lane % GLp)*VEC.
template <int VEC, int GL, int NCH>
__device__ __forceinline__ void hub_sum(int first, int nch, int C, const float* __restrict__ partials,
                                        float (&hs)[NCH][VEC]) {
  constexpr int GLp = pow2_ceil(GL);
  constexpr int G = kWave / GLp;
  static_assert(NCH == 1 || GLp == GL, "several column passes need power-of-two row lanes");
  const int lane = threadIdx.x & 63;
  const int g = lane / GLp, gl = lane % GLp;
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int cc = (ch * GLp + gl) * VEC;
    const bool live = cc < C;
#pragma unroll
    for (int t = 0; t < VEC; ++t) hs[ch][t] = 0.f;
#pragma unroll 4
    for (int c = g; c < nch; c += G) {
      float v[VEC];
      if (live) {
        load_vec<VEC>(partials + (int64_t)(first + c) * C + cc, v);
      } else {
#pragma unroll
        for (int t = 0; t < VEC; ++t) v[t] = 0.f;
      }
#pragma unroll
      for (int t = 0; t < VEC; ++t) hs[ch][t] += v[t];
    }
#pragma unroll
    for (int o = GLp; o < kWave; o <<= 1)
#pragma unroll
      for (int t = 0; t < VEC; ++t) hs[ch][t] += __shfl_xor(hs[ch][t], o);
  }
}

// Memory order of the arrival ticket.  The partials are stored write-through and
// drained (s_waitcnt vmcnt(0)) before the ticket, which is what an agent-scope
// release orders at the ISA level; GNPDE_HUB_RELEASE=1 builds the ticket as a
// formal C++ release as well (it adds buffer_wbl2 sc1: a write-back of every
// dirty line of the XCD's L2 before each chunk's ticket).
#ifndef GNPDE_HUB_RELEASE
#define GNPDE_HUB_RELEASE 0
#endif
constexpr int kHubTicketOrder = GNPDE_HUB_RELEASE ? __ATOMIC_RELEASE : __ATOMIC_RELAXED;

// Chunk waves whose write-through partial stores are issued: drain them; each
// row slot holding a hub chunk takes an arrival ticket on its hub's plan entry
// (heavy[h].w, an agent-scope atomic; hubs found by a binary search of the
// ascending first slots); every slot whose chunk arrived last then has its hub
// row summed by the whole wavefront (hub_sum, after an acquire; the ticket is
// reset to 0 for the next launch on this plan), and the slot's owner lanes take
// the row (erow) and its sums (acc) for the kernel's one epilogue.  Called by
// all 64 lanes; `chunk`, `slot` are per slot.  Returns whether this lane now
// owns a hub row.
template <int VEC, int GL, int SL, int RPW, int NCH>
__device__ __forceinline__ bool hub_claim(int4* heavy, int n_heavy, bool chunk, int slot, int C,
                                          const float* partials, int rs, int g, int gl, int& erow,
                                          float (&acc)[NCH][VEC]) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int lane = threadIdx.x & 63;
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
    if (lane % SL == 0) {
      const int t = __hip_atomic_fetch_add(&heavy[lo].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
      won = t == heavy[lo].z - 1;
    }
  }
  bool mine = false;
  for (int s = 0; s < RPW; ++s) {
    if (__shfl(won, s * SL)) {  // wave-uniform
      const int h = __shfl(lo, s * SL);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const int4 hv = heavy[h];
      float hs[NCH][VEC];
      hub_sum<VEC, GL, NCH>(uniform(hv.y), uniform(hv.z), C, partials, hs);
      // the slot's lane gl takes the sums of its columns from lane gl (group 0 holds every column)
      const bool take = rs == s && g == 0;
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
        for (int t = 0; t < VEC; ++t) {
          const float v = (GL == kWave) ? hs[ch][t] : __shfl(hs[ch][t], gl);
          acc[ch][t] = take ? v : acc[ch][t];
        }
      if (take) {
        erow = uniform(hv.x);
        mine = true;
      }
      if (lane == 0) __hip_atomic_store(&heavy[h].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
  return mine;
}

// The hub combine of the flash kernels (flash.hip; agg_kernel uses hub_claim): each row slot of the wavefront that holds a
// hub chunk takes its own ticket (its first lane); every slot whose chunk
// arrived last is then combined by the WHOLE wavefront, one slot after the
// other (hub_combine over 64 lanes: the same sums, in the same order, as
// agg_fixup_kernel).  Called by all 64 lanes; `chunk` is per slot.
template <int VEC, int GL, int SL, int RPW, int STG, class T>
__device__ __forceinline__ void hub_arrive_slots(int4* heavy, int n_heavy, bool chunk, int slot, int C,
                                                 const Epi& ep, const float* partials) {
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  const int lane = threadIdx.x & 63;
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
    if (lane % SL == 0) {
      const int t = __hip_atomic_fetch_add(&heavy[lo].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
      won = t == heavy[lo].z - 1;
    }
  }
#pragma unroll
  for (int s = 0; s < RPW; ++s) {
    if (__shfl(won, s * SL)) {  // wave-uniform
      const int h = __shfl(lo, s * SL);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      const int4 hv = heavy[h];
      hub_combine<VEC, pow2_ceil(GL), STG, T>(uniform(hv.x), uniform(hv.y), uniform(hv.z), C, ep, partials);
      if (lane == 0) __hip_atomic_store(&heavy[h].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
  }
}

// The folded dense output's crossing flag and coefficients (dense_coefs), formed ahead of
// the launch whose stage asks for them (ABI 8: dense_tab without dense_out) for the step's
// last launch.  A launch of its own: the same branch at the top of the aggregation kernel
// cost every instantiation (BLEND's fp32 rk4 step 0.556 -> 0.583 ms).
static __global__ __launch_bounds__(64) void dense_coef_kernel(gnpde_stage_epilogue_t st) {
  if (threadIdx.x == 0) dense_coefs(st, st.dense_tab);
}

// ------------------------------------------------------------------ aggregation kernel
// Lane layout: RPW row slots of SL = 64/RPW lanes per wavefront (one plan item
// each); inside a slot lane = g*GL + gl: G = SL/GL edges are gathered side by
// side, each by a group of GL lanes covering the C columns with VEC-wide loads
// (NCH column passes); U edges per group are in flight per iteration.  The
// epilogue operands (x_r, x0_r, stage inputs) are loaded before the gathers
// when NCH <= 2 (PRE) so their latency overlaps the aggregation.  Hub rows are
// combined in-launch by the chunk that arrives last (hub_claim), and run
// through the same epilogue as whole rows.
template <int VEC, int GL, int NCH, int U, int RPW, int STG, class WP, class T = float>
__global__ __launch_bounds__(256) void agg_kernel(const int4* __restrict__ items, int n_items, int4* heavy,
                                                   int n_heavy, const int* __restrict__ col, WP wp, int C, Epi ep,
                                                   float* __restrict__ partials) {
  constexpr int SL = kWave / RPW;
  constexpr int G = SL / GL;
  static_assert((SL & (SL - 1)) == 0 || G == 1, "non-power-of-two row slots hold one edge group");
  constexpr bool PRE = NCH <= 2;
  const int lane = threadIdx.x & 63;
  const int rs = lane / SL, sl = lane % SL;
  const int g = sl / GL, gl = sl % GL;
  const int wid = uniform(xcd_block(ep.xcd_remap) * kWavesPerBlock + (threadIdx.x >> 6));
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  // RPW = 3 (SL = 21): lane 63 is in no slot
  const bool live = item < n_items && rs < RPW;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const bool owner = live && slot < 0 && g == 0;

  EpiPre<VEC, T, STG> pre[PRE ? NCH : 1];
  if constexpr (PRE) {
    if (owner) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int cc = (ch * GL + gl) * VEC;
        if (cc < C) epi_prefetch<VEC, STG, T>(ep, row, cc, pre[ch]);
      }
    }
  }

  float acc[NCH][VEC];
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
    for (int t = 0; t < VEC; ++t) acc[ch][t] = 0.f;

  for (int e0 = beg; e0 < end; e0 += SL) {
    const int n = min(SL, end - e0);
    int mc = 0;
    typename WP::Raw raw{};
    if (sl < n) {
      mc = col[e0 + sl];
      raw = wp.load(row, e0 + sl, mc);
    }
    float mw = 0.f;
    for (int j = 0; j < n; j += G * U) {
      Packed<VEC, T> v[U][NCH];  // gathered row slices in storage form (bf16: half the registers)
      float ww[U];
      int srcl[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u * G + g;
        const int src = rs * SL + (jj < n ? jj : 0);
        srcl[u] = src;
        const int c = __shfl(mc, src);
        const T* __restrict__ xr = as_t<T>(ep.x) + (int64_t)c * ep.ldx;
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int cc = (ch * GL + gl) * VEC;
          if (jj < n && cc < C) {
            load_packed<VEC>(xr + cc, v[u][ch]);
          } else {
#pragma unroll
            for (int t = 0; t < Packed<VEC, T>::W; ++t) v[u][ch].d[t] = 0u;
          }
        }
      }
      // the weights of this batch of edges, finished while its first gathers are in flight
      if (j == 0 && sl < n) mw = wp.finish(row, raw);
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u * G + g;
        const float wsl = __shfl(mw, srcl[u]);
        ww[u] = jj < n ? wsl : 0.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
          for (int t = 0; t < VEC; ++t) acc[ch][t] = fmaf(ww[u], unpack(v[u][ch], t), acc[ch][t]);
    }
  }
  // combine the G edge groups of each slot
#pragma unroll
  for (int o = GL; o < SL; o <<= 1)
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch)
#pragma unroll
      for (int t = 0; t < VEC; ++t) acc[ch][t] += __shfl_xor(acc[ch][t], o);

  // The row whose epilogue this lane runs: its own (an owner lane of a whole
  // row), or a hub row whose chunk arrived last in this wavefront (hub_claim);
  // ONE epilogue below serves both, so the hub combine adds no second copy of
  // the (wide) epilogue to the kernel's register allocation.
  int erow = row;
  bool fin = live && slot < 0 && g == 0;
  bool hub = false;
  if (n_heavy > 0) {  // hub chunks of any slot combined in-launch
    const bool chunk = live && slot >= 0;
    int anyc = 0;
#pragma unroll
    for (int s = 0; s < RPW; ++s) anyc |= __shfl((int)chunk, s * SL);
    if (anyc) {  // wave-uniform
      if (chunk && g == 0) {
        const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
#pragma unroll
        for (int ch = 0; ch < NCH; ++ch) {
          const int cc = (ch * GL + gl) * VEC;
          buf_store_wt<VEC>(rp, cc < C ? (uint32_t)(((int64_t)slot * C + cc) * 4) : kBufNone, acc[ch]);
        }
      }
      hub = hub_claim<VEC, GL, SL, RPW, NCH>(heavy, n_heavy, chunk, slot, C, partials, rs, g, gl, erow, acc);
      fin = fin || hub;
    }
  } else if (live && slot >= 0 && g == 0) {  // chunk partials of a later agg_fixup_kernel
#pragma unroll
    for (int ch = 0; ch < NCH; ++ch) {
      const int cc = (ch * GL + gl) * VEC;
      if (cc < C) store_vec<VEC>(partials + (int64_t)slot * C + cc, acc[ch]);
    }
    return;
  }
  if (!fin) return;
  if constexpr (PRE) {  // a hub row's epilogue operands were not prefetched
    if (hub) {
#pragma unroll
      for (int ch = 0; ch < NCH; ++ch) {
        const int cc = (ch * GL + gl) * VEC;
        if (cc < C) epi_prefetch<VEC, STG, T>(ep, erow, cc, pre[ch]);
      }
    }
  }
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart[2] = {0.0, 0.0};
#pragma unroll
  for (int ch = 0; ch < NCH; ++ch) {
    const int cc = (ch * GL + gl) * VEC;
    if (cc < C) {
      if constexpr (PRE)
        epi_finish<VEC, STG, T>(ep, erow, cc, acc[ch], a, b, pre[ch], dpart);
      else
        epilogue_store<VEC, STG, T>(ep, erow, cc, acc[ch], a, b, dpart);
    }
  }
  // the row's owner lanes (g == 0: lanes [rs*SL, rs*SL + GL)) are all here
  if constexpr (stage_rowsum<STG, T>()) {
    const double* prev = nullptr;
    if constexpr (PRE && stage_dot<STG>() && GNPDE_DOT_PRE) prev = &pre[0].dprev;
    epi_rowsums<GL, STG, T>(ep, erow, dpart, rs * SL, gl == 0, prev);
  }
}

// Hub rows combined after the aggregation launch (GNPDE_HUB_FIXUP=1): one wavefront per hub.
template <int VEC, int GL, int STG, class T = float>
__global__ __launch_bounds__(256) void agg_fixup_kernel(const int4* __restrict__ heavy, int n_heavy, int C, Epi ep,
                                                         const float* __restrict__ partials) {
  const int wid = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (wid >= n_heavy) return;
  const int4 hv = heavy[wid];
  hub_combine<VEC, pow2_ceil(GL), STG, T>(uniform(hv.x), uniform(hv.y), uniform(hv.z), C, ep, partials);
}

// Experiment builds only (make EXPERIMENTS=1 defines GNPDE_EXPERIMENTS=1; the
// product library has none of this): GNPDE_HUB_FIXUP=1 combines hub rows in a
// separate agg_fixup_kernel launch instead of inside the aggregation, and
// GNPDE_AGG_VARIANT selects alternative lane geometries (the round-2 A/B sweeps
// recorded in DESIGN.md §6-§7).
bool hub_inlaunch();
int agg_variant();

template <int VEC, int GL, int NCH, int U, int RPW, class WP, class T = float>
static int launch_agg_cfg(const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                          const WP& wp, int C, const Epi& ep, float* partials, hipStream_t s) {
  const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * RPW);
  // hub rows are combined in the launch (hub_claim)
  bool inlaunch = true;
  if constexpr (GNPDE_EXPERIMENTS) inlaunch = hub_inlaunch();
  const int nh = inlaunch ? (int)n_heavy : 0;
  // single-output stages without dot terms (every forward gnpde.integrator step) get the
  // leaner instantiation: 56-60 VGPRs, 8 waves per SIMD; the dot terms of the adjoint
  // stages alone cost the general one 40+ VGPRs (fused rk4 K1 92.9 -> 107 us at 4 waves)
  int stg = epi_stage_kind(ep);
  if (ep.has_stage && ep.st.dense_tab && !ep.st.dense_out) {  // the step's dense-output coefficients
    dense_coef_kernel<<<1, kWave, 0, s>>>(ep.st);
    GNPDE_LAUNCH_CHECK();
  }
  if (n_items > 0) {
    // the one-output adjoint stages: fp32 plain weights only (the transposed aggregation)
    if (stg == 3 && !(std::is_same<WP, PlainWeights>::value && sizeof(T) == 4)) stg = 2;
    if (stg == 4) {
      // the adaptive solvers' wide epilogue: plain weights only (the Laplacian RHS and
      // precomputed attention weights); the callers apply it after the other policies
      if constexpr (std::is_same<WP, PlainWeights>::value) {
        if (ep.st.dense_out)  // + the step's folded dense output (ABI 8)
          agg_kernel<VEC, GL, NCH, U, RPW, 5, PlainWeights, T><<<grid, kBlock, 0, s>>>(
              items, (int)n_items, heavy, nh, col, as_plain(wp), C, ep, partials);
        else
          agg_kernel<VEC, GL, NCH, U, RPW, 4, PlainWeights, T><<<grid, kBlock, 0, s>>>(
              items, (int)n_items, heavy, nh, col, as_plain(wp), C, ep, partials);
      } else {
        set_error("rhs: the wide (adaptive-solver) stage epilogue is fused with plain weights only; "
                  "apply it with gnpde_stage_apply_*");
        return GNPDE_EUNSUPPORTED;
      }
    } else if (stg == 3)
      agg_kernel<VEC, GL, NCH, U, RPW, 3, PlainWeights, float><<<grid, kBlock, 0, s>>>(
          items, (int)n_items, heavy, nh, col, as_plain(wp), C, ep, partials);
    else if (stg == 1)
      agg_kernel<VEC, GL, NCH, U, RPW, 1, WP, T><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, wp, C, ep,
                                                                          partials);
    else if (stg == 2)
      agg_kernel<VEC, GL, NCH, U, RPW, 2, WP, T><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, wp, C, ep,
                                                                          partials);
    else
      agg_kernel<VEC, GL, NCH, U, RPW, 0, WP, T><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, wp, C, ep,
                                                                          partials);
    GNPDE_LAUNCH_CHECK();
  }
  if constexpr (GNPDE_EXPERIMENTS) {
    const unsigned gfix = (unsigned)ceil_div(n_heavy, kWavesPerBlock);
    if (!inlaunch && n_heavy > 0) {
      if (stg == 3 || stg == 4) stg = 2;
      if (stg == 1)
        agg_fixup_kernel<VEC, GL, 1, T><<<gfix, kBlock, 0, s>>>(heavy, (int)n_heavy, C, ep, partials);
      else if (stg == 2)
        agg_fixup_kernel<VEC, GL, 2, T><<<gfix, kBlock, 0, s>>>(heavy, (int)n_heavy, C, ep, partials);
      else
        agg_fixup_kernel<VEC, GL, 0, T><<<gfix, kBlock, 0, s>>>(heavy, (int)n_heavy, C, ep, partials);
      GNPDE_LAUNCH_CHECK();
    }
  }
  return GNPDE_OK;
}

// The lane geometry of a row width (lanes = ceil(C / VEC)), measured per width in
// round 1-2 (profiles/r02b_stripe_sweep.jsonl, r02b_layout_ab.jsonl).
template <int VEC, class WP, class T = float>
static int launch_agg_vec(const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                          const WP& wp, int C, const Epi& ep, float* partials, hipStream_t s) {
  const int lanes = (int)ceil_div(C, VEC);
#define GNPDE_AGG(GL, NCH, U, RPW) \
  launch_agg_cfg<VEC, GL, NCH, U, RPW, WP, T>(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, s)
  const int var = GNPDE_EXPERIMENTS ? agg_variant() : 0;
  if constexpr (GNPDE_EXPERIMENTS) {
    switch (var) {
      case 6:  // twice the gathers in flight per edge group
        if (lanes <= 4) return GNPDE_AGG(4, 1, 8, 8);
        if (lanes <= 8) return GNPDE_AGG(8, 1, 8, 4);
        if (lanes <= 16) return GNPDE_AGG(16, 1, 8, 2);
        break;
      case 8:  // half the rows per wavefront, four edge groups per row
        if (lanes <= 4) return GNPDE_AGG(4, 1, 4, 4);
        if (lanes <= 8) return GNPDE_AGG(8, 1, 4, 2);
        if (lanes <= 16) return GNPDE_AGG(16, 1, 4, 1);
        break;
      // narrow stripes (the column layout at 4-8 ranks): edge groups per row x unroll
      case 20: if (lanes <= 4) return GNPDE_AGG(4, 1, 8, 4); if (lanes <= 8) return GNPDE_AGG(8, 1, 4, 4); break;
      case 21: if (lanes <= 4) return GNPDE_AGG(4, 1, 2, 4); if (lanes <= 8) return GNPDE_AGG(8, 1, 8, 2); break;
      case 22: if (lanes <= 4) return GNPDE_AGG(4, 1, 4, 8); if (lanes <= 8) return GNPDE_AGG(8, 1, 4, 2); break;
      case 23: if (lanes <= 4) return GNPDE_AGG(4, 1, 8, 2); if (lanes <= 8) return GNPDE_AGG(8, 1, 2, 4); break;
      case 24: if (lanes <= 4) return GNPDE_AGG(4, 1, 4, 2); if (lanes <= 8) return GNPDE_AGG(8, 1, 8, 8); break;
      case 2: if (lanes > 16 && lanes <= 32) return GNPDE_AGG(32, 1, 2, 1); break;
      case 3:
        if (lanes > 16 && lanes <= 32) return GNPDE_AGG(32, 1, 8, 1);
        if (lanes > 32 && lanes <= 64) return GNPDE_AGG(64, 1, 8, 1);
        break;
      case 4: if (lanes > 16 && lanes <= 32) return GNPDE_AGG(32, 1, 4, 1); break;
      default: break;
    }
  }
  // Narrow rows (the column stripes of gnpde.dist at 2-8 GPUs: G-arxiv C = 128 / 8 = 16
  // floats = 4 lanes; G-rmat 256 / 8 = 32 floats = 8 lanes): several rows per
  // wavefront with 2-4 edges side by side per row slot, instead of one row per
  // wavefront idling 3/4 of a 16-lane group (G-arxiv rk4 step at 16 / 32 / 64 columns:
  // 0.133 / 0.152 / 0.243 ms against 0.266 / 0.270 / 0.296 with one row per wavefront).
  // A state far beyond the Infinity Cache (G-rmat stripes: 2M rows x 32-64 columns) is
  // gathered from HBM, where more independent rows per wavefront win (G-rmat rk4 step at
  // 32 / 64 columns 2.06 / 3.67 ms against 2.56 / 4.52); a cache-resident one (G-arxiv
  // stripes) prefers several edge groups per row (0.149 / 0.124 ms at 32 / 16 columns
  // against 0.283 / 0.318).
  // (plain weights only: the attention-weight policies take the 16-lane geometry for
  // narrow rows, which keeps the library's instantiation count down)
  if constexpr (std::is_same<WP, PlainWeights>::value) {
    if (var != 5) {
      if (n_items * (int64_t)C * (int64_t)sizeof(T) > (int64_t)(96 << 20)) {
        if (lanes <= 4) return GNPDE_AGG(4, 1, 4, 16);
        if (lanes <= 8) return GNPDE_AGG(8, 1, 4, 8);
        if (lanes <= 16) return GNPDE_AGG(16, 1, 4, 4);
      }
      if (lanes <= 4) return GNPDE_AGG(4, 1, 4, 4);
      if (lanes <= 8) return GNPDE_AGG(8, 1, 8, 4);
      if (lanes <= 16) return GNPDE_AGG(16, 1, 4, 2);
    }
  }
  if (lanes <= 16) return GNPDE_AGG(16, 1, 4, 1);
  if constexpr (sizeof(T) == 2 && VEC == 8) {
    // bf16 rows of 129-168 columns (BLEND: C = 162 padded to 168 = 21 lanes of 16 B):
    // three rows per wavefront, 63 of 64 lanes busy
    if (lanes > 16 && lanes <= 21) return GNPDE_AGG(21, 1, 4, 3);
  }
  // two rows per wavefront (fp32 C = 128 and bf16 rows of 17-32 lanes): with the
  // plan's items longest first, G-arxiv rk4 bench 9,301 against 8,643 RHS/s with
  // one row per wavefront
  if (lanes <= 32) return GNPDE_AGG(32, 1, 4, 2);
  if (lanes <= 64) return GNPDE_AGG(64, 1, 4, 1);
  if (lanes <= 128) return GNPDE_AGG(64, 2, 2, 1);
  if (lanes <= 256) return GNPDE_AGG(64, 4, 2, 1);
  if (lanes <= 512) return GNPDE_AGG(64, 8, 1, 1);
#undef GNPDE_AGG
  set_error("aggregate: C=%d too wide (max %d)", C, 512 * VEC);
  return GNPDE_EUNSUPPORTED;
}

// Widest vector (elements per lane: 4, 2 or 1 floats; 8, 4, 2 or 1 bf16) every
// operand of the aggregation and its epilogue allows: C, the leading dimensions
// and all pointers must agree.
// Experiment knob (not part of the ABI contract): GNPDE_BF16_VEC caps the
// elements per lane of bf16 rows (default 4 = 8-byte gathers; 8 = 16-byte).
int bf16_vec_cap();

// bf16 rows are sized to land in 17-32 lanes, the two-rows-per-wavefront
// geometry (launch_agg_vec): 8-byte gathers up to 128 columns, 16-byte gathers
// for 129-256 columns (G-arxiv, items longest first: C = 128 58 us against 77-96;
// BLEND C = 168 77 us against 93-122, 0.353-0.361 ms per rk4 step against 0.402).
template <class T = float>
inline int epi_vec_width(const Epi& ep, int64_t C, const void* partials) {
  const int kMax = sizeof(T) == 2 ? ((C > 128 && C <= 256 && bf16_vec_cap() >= 4) ? 8 : bf16_vec_cap())
                                  : 16 / (int)sizeof(T);
  for (int v = kMax; v > 1; v >>= 1) {
    const size_t bytes = (size_t)v * sizeof(T);
    auto al = [&](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0; };
    bool ok = C % v == 0 && ep.ldx % v == 0 && ep.ldf % v == 0 && al(ep.x);
    if (ep.flags & GNPDE_ADD_SOURCE) ok = ok && ep.ldx0 % v == 0 && al(ep.x0);
    if (ep.has_stage) {
      ok = ok && al(ep.st.f_out);
      for (int i = 0; i < ep.st.n_out; ++i) {
        ok = ok && al(ep.st.o[i].out) && al(ep.st.o[i].base);
      }
      for (int j = 0; j < ep.st.nk; ++j) ok = ok && al(ep.st.k[j]);
      if (ep.st.err_rows) ok = ok && al(ep.st.err.base) && al(ep.st.err_y0);
    } else {
      ok = ok && al(ep.f);
    }
    // fp32 partials are written with the same lane slices: v floats per lane (16-B pieces at most)
    ok = ok && (partials == nullptr || (reinterpret_cast<uintptr_t>(partials) % std::min<size_t>(16, 4 * v)) == 0);
    if (ok) return v;
  }
  return 1;
}

template <class WP, class T = float>
static int launch_agg(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                      const int32_t* col, const WP& wp, int64_t C, const Epi& ep, float* partials, hipStream_t s) {
  const int4* it = reinterpret_cast<const int4*>(items);
  int4* hv = reinterpret_cast<int4*>(heavy);
  const int c = (int)C;
  switch (epi_vec_width<T>(ep, C, partials)) {
    case 8:
      if constexpr (sizeof(T) == 2) return launch_agg_vec<8, WP, T>(it, n_items, hv, n_heavy, col, wp, c, ep, partials, s);
      [[fallthrough]];
    case 4: return launch_agg_vec<4, WP, T>(it, n_items, hv, n_heavy, col, wp, c, ep, partials, s);
    case 2: return launch_agg_vec<2, WP, T>(it, n_items, hv, n_heavy, col, wp, c, ep, partials, s);
    default: return launch_agg_vec<1, WP, T>(it, n_items, hv, n_heavy, col, wp, c, ep, partials, s);
  }
}

}  // namespace gnpde
