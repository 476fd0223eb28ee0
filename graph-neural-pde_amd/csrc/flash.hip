// flash.hip — the per-edge scaled_dot attention RHS under source-grouped
// softmax (attention_norm_idx 0, upstream GRAND's default transformer RHS) as
// ONE aggregation pass: the softmax group of an edge is its source, which is
// the row the aggregation sums into, so each wavefront row slot scores the
// edges it gathers and keeps an online (running max, rescaled sum) softmax per
// head while it accumulates (the flash-attention recurrence on a graph row).
// No [nnz] weight array, no separate softmax launch.  Reference:
//   SpGraphTransAttentionLayer.forward  src/function_transformer_attention.py:218-266
//     (q = Q x, k = K x, prods = q_src . k_dst / sqrt(dk) — upstream's per-edge score)
//   utils.softmax (groups = edge_index[0])  src/utils.py:116-127
//   multiply_attention (head mean, A x)     src/function_transformer_attention.py:33-41
//   ODEFuncTransformerAtt.forward            :44-59 (f = a (A x - x) [+ b x0])
//
// Per row r with edges e -> c_e, head h:
//   s_e,h = q_r,h . k_c,h / sqrt(dk)
//   M_h = max_e s_e,h,  L_h = sum_e exp(s_e,h - M_h),  acc_h = sum_e exp(s_e,h - M_h) x_c
//   ax_r = (1/H) sum_h acc_h / (L_h + 1e-16)
// which is sum_e w_e x_c with the reference's w_e = mean_h softmax_e,h.  The
// running (M, L, acc) of a row slot are rescaled by exp(M_old - M_new) once per
// batch of U edges.  Scores and exponentials use base 2 (s * log2(e) and
// v_exp_f32), 1-2 ulp from expf.
//
// Lane layout (row slots of GL = 16 / 32 / 64 lanes, C <= 4 GL, 4 floats per lane
// as in K1): the q . k product of an edge is formed in every 16-lane DPP row of
// the slot — lane l of a row holds q / k elements [4 (l mod att/4), +4) — and
// reduced over the dk/4 lanes of a head by quad permutes and row mirrors; each
// head's score then reaches the whole row by a row_newbcast.  The k slice of an
// edge is loaded with the same column index as its x row, so both gathers are in
// flight together (one memory round trip per batch, as K1).
//
// Hub rows (more than `chunk` edges) are split into chunk items as in K1; a
// chunk stores its running state (acc_h, M_h, L_h) write-through to its slot
// and takes an arrival ticket on the hub's plan entry; the last chunk merges
// the slots in fixed order (deterministic, no float atomics) and runs the
// epilogue.
#include "aggregate.hpp"
#include "rhs_host.hpp"

namespace gnpde {

constexpr float kLog2e = 1.4426950408889634f;

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

// sum over the S = dk/4 lanes of a head (S in {1, 2, 4, 8, 16}, aligned inside a 16-lane row)
__device__ __forceinline__ float head_reduce(float v, int S) {
  if (S >= 2) v += dpp_mov<0xB1>(v);   // quad_perm [1,0,3,2]
  if (S >= 4) v += dpp_mov<0x4E>(v);   // quad_perm [2,3,0,1]
  if (S >= 8) v += dpp_mov<0x141>(v);  // row_half_mirror
  if (S >= 16) v += dpp_mov<0x140>(v); // row_mirror
  return v;
}

// lane l of a 16-lane row: score of head h (lanes [h S, (h+1) S) of the row) to every lane of the row
template <int MAXH>
__device__ __forceinline__ void heads_bcast(float v, int S, float (&s)[MAXH]) {
#define GNPDE_NB(H)                                                  \
  if constexpr (MAXH > H) {                                          \
    if (S == 1) s[H] = dpp_mov<0x150 + H>(v);                        \
    else if (S == 2) s[H] = dpp_mov<0x150 + ((2 * H) & 15)>(v);      \
    else if (S == 4) s[H] = dpp_mov<0x150 + ((4 * H) & 15)>(v);      \
    else if (S == 8) s[H] = dpp_mov<0x150 + ((8 * H) & 15)>(v);      \
    else s[H] = v;                                                   \
  }
  GNPDE_NB(0)
  GNPDE_NB(1)
  GNPDE_NB(2)
  GNPDE_NB(3)
#undef GNPDE_NB
}

struct DotArgs {
  const float* __restrict__ q;  // [R, ldqk]: q_r at q + r*ldqk, att = H*dk floats
  const float* __restrict__ k;
  int64_t ldqk;
  int H, S;       // heads, lanes per head (dk / 4)
  int qlanes;     // att / 4: lanes of a row holding distinct slices
  float scale;    // log2(e) / sqrt(dk)
  int ps;         // floats per partial slot: H*C acc, then M[H], L[H] (rounded up to 4)
};

__device__ __forceinline__ int64_t slice_off(const DotArgs& da, int lane) {
  return (int64_t)((lane & 15) % da.qlanes) * 4;
}

// Merge the chunk slots of hub row `row` (first .. first+nch-1) and run the
// epilogue: per head M = max of the chunk maxima, then acc and L scaled by
// exp(M_c - M), summed in chunk order.  Lanes cover the columns (C <= 256).
template <int MAXH, int STG>
__device__ __forceinline__ void flash_hub_combine(int row, int first, int nch, int C, const DotArgs& da,
                                                  const Epi& ep, const float* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int cc = lane * 4;
  const bool live = cc < C;
  const int H = da.H;
  float M[MAXH], L[MAXH], acc[MAXH][4];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = 0.f;
  }
  for (int c = 0; c < nch; ++c) {
    const float* p = partials + (int64_t)(first + c) * da.ps;
#pragma unroll
    for (int h = 0; h < MAXH; ++h)
      if (h < H) M[h] = fmaxf(M[h], p[H * C + h]);
  }
  for (int c = 0; c < nch; ++c) {
    const float* p = partials + (int64_t)(first + c) * da.ps;
#pragma unroll
    for (int h = 0; h < MAXH; ++h) {
      if (h < H) {
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
  }
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    if (h < H) {
      const float r = 1.0f / (L[h] + kSoftmaxEps);
#pragma unroll
      for (int t = 0; t < 4; ++t) ax[t] = fmaf(acc[h][t], r, ax[t]);
    }
  }
  const float inv_h = 1.0f / (float)H;
#pragma unroll
  for (int t = 0; t < 4; ++t) ax[t] *= inv_h;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (live) epilogue_store<4, STG, float>(ep, row, cc, ax, a, b, &dpart);
  if constexpr (STG >= 2)
    if (ep.st.dot_rows) epi_dot_store<64>(ep, row, dpart, lane == 0);  // every lane of the wave (convergent)
}

template <int GL, int U, int MAXH, int STG>
__global__ __launch_bounds__(256) void flash_agg_kernel(const int4* __restrict__ items, int n_items, int4* heavy,
                                                         int n_heavy, const int* __restrict__ col, DotArgs da, int C,
                                                         Epi ep, float* __restrict__ partials) {
  constexpr int RPW = kWave / GL;
  constexpr int SL = GL;
  const int lane = threadIdx.x & 63;
  const int rs = lane / SL, gl = lane % SL;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  const int item = wid * RPW + rs;
  if (wid * RPW >= n_items) return;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int row = it.x, beg = it.y, end = it.z, slot = it.w;
  const int cc = gl * 4;
  const bool colv = cc < C;
  const int H = da.H;

  EpiPre<4, float, stage_nout<STG>()> pre;
  if (live && slot < 0 && colv) epi_prefetch<4, STG, float>(ep, row, cc, pre);
  const int64_t ko = slice_off(da, lane);
  float qv[4];
  load_vec<4>(da.q + (int64_t)row * da.ldqk + ko, qv);

  float M[MAXH], L[MAXH], acc[MAXH][4];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t) acc[h][t] = 0.f;
  }

  // every lane runs the loop the same number of times (the DPP steps need the
  // whole row): the slot with the longest item sets the trip count
  int len = end - beg;
  int nmax = len;
#pragma unroll
  for (int o = SL; o < kWave; o <<= 1) nmax = max(nmax, __shfl_xor(nmax, o));
  for (int e0 = 0; e0 < nmax; e0 += SL) {
    const int n = min(SL, len - e0);  // may be <= 0 for a short slot
    int mc = 0;
    if (gl < n) mc = col[beg + e0 + gl];
    const int nn = min(SL, nmax - e0);
    for (int j = 0; j < nn; j += U) {
      float xv[U][4], kv[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int jj = j + u;
        const bool ok = jj < n;
        const int c = __shfl(mc, rs * SL + (jj < SL ? jj : 0));
        if (ok && colv) {
          load_vec<4>(ep.x + (int64_t)c * ep.ldx + cc, xv[u]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) xv[u][t] = 0.f;
        }
        if (ok) {
          load_vec<4>(da.k + (int64_t)c * da.ldqk + ko, kv[u]);
        } else {
#pragma unroll
          for (int t = 0; t < 4; ++t) kv[u][t] = 0.f;
        }
      }
      float s[U][MAXH];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        float d = 0.f;
#pragma unroll
        for (int t = 0; t < 4; ++t) d = fmaf(qv[t], kv[u][t], d);
        d = head_reduce(d, da.S) * da.scale;  // full-wave DPP
        heads_bcast<MAXH>(d, da.S, s[u]);
        if (j + u >= n) {
#pragma unroll
          for (int h = 0; h < MAXH; ++h) s[u][h] = -INFINITY;
        }
      }
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        if (h < H) {
          float mb = M[h];
#pragma unroll
          for (int u = 0; u < U; ++u) mb = fmaxf(mb, s[u][h]);
          if (mb != -INFINITY) {  // some edge of the batch is live for this slot
            const float corr = __builtin_amdgcn_exp2f(M[h] - mb);  // exp2(-inf) = 0 on the first batch
            float p[U];
            float ls = 0.f;
#pragma unroll
            for (int u = 0; u < U; ++u) {
              p[u] = __builtin_amdgcn_exp2f(s[u][h] - mb);
              ls += p[u];
            }
            L[h] = fmaf(L[h], corr, ls);
#pragma unroll
            for (int t = 0; t < 4; ++t) {
              float a = acc[h][t] * corr;
#pragma unroll
              for (int u = 0; u < U; ++u) a = fmaf(p[u], xv[u][t], a);
              acc[h][t] = a;
            }
            M[h] = mb;
          }
        }
      }
    }
  }

  // a chunk of a hub row: store the running state, merge in-launch (last arrival)
  const bool chunk = live && slot >= 0;
  if (n_heavy > 0) {
    int anyc = 0;
#pragma unroll
    for (int s = 0; s < RPW; ++s) anyc |= __shfl((int)chunk, s * SL);
    if (anyc) {  // wave-uniform
      const __amdgpu_buffer_rsrc_t rp = buf_rsrc(partials);
      const int64_t base = (int64_t)(chunk ? slot : 0) * da.ps;
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        if (h < H) {
          buf_store_wt<4>(rp, (chunk && colv) ? (uint32_t)((base + h * C + cc) * 4) : kBufNone, acc[h]);
          float ml[1] = {M[h]};
          buf_store_wt<1>(rp, (chunk && gl == 0) ? (uint32_t)((base + H * C + h) * 4) : kBufNone, ml);
          ml[0] = L[h];
          buf_store_wt<1>(rp, (chunk && gl == 0) ? (uint32_t)((base + H * C + H + h) * 4) : kBufNone, ml);
        }
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
        if (gl == 0) {
          const int t = __hip_atomic_fetch_add(&heavy[lo].w, 1, kHubTicketOrder, __HIP_MEMORY_SCOPE_AGENT);
          won = t == heavy[lo].z - 1;
        }
      }
#pragma unroll
      for (int s = 0; s < RPW; ++s) {
        if (__shfl(won, s * SL)) {  // wave-uniform
          const int hh = __shfl(lo, s * SL);
          __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
          const int4 hv = heavy[hh];
          flash_hub_combine<MAXH, STG>(uniform(hv.x), uniform(hv.y), uniform(hv.z), C, da, ep, partials);
          if (lane == 0) __hip_atomic_store(&heavy[hh].w, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
      }
      if (chunk) return;
    }
  }
  if (!live || slot >= 0) return;
  float ax[4] = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    if (h < H) {
      const float r = 1.0f / (L[h] + kSoftmaxEps);
#pragma unroll
      for (int t = 0; t < 4; ++t) ax[t] = fmaf(acc[h][t], r, ax[t]);
    }
  }
  const float inv_h = 1.0f / (float)H;
#pragma unroll
  for (int t = 0; t < 4; ++t) ax[t] *= inv_h;
  const float a = (ep.flags & GNPDE_EPI_RHS) ? epi_alpha(ep) : 1.f;
  const float b = (ep.flags & GNPDE_ADD_SOURCE) ? *ep.beta : 0.f;
  double dpart = 0.0;
  if (colv) epi_finish<4, STG, float>(ep, row, cc, ax, a, b, pre, &dpart);
  if constexpr (STG >= 2)
    if (ep.st.dot_rows) {
      // the slot's lanes hold the row's partial dot terms: a fixed xor tree over the slot
#pragma unroll
      for (int o = 1; o < SL; o <<= 1) dpart += __shfl_xor(dpart, o);
      if (gl == 0) {
        double* d = ep.st.dot_rows + row;
        const double v = ep.st.dot_coef * dpart;
        *d = ep.st.dot_accumulate ? *d + v : v;
      }
    }
}

template <int GL, int MAXH>
static int launch_flash_h(const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                          const DotArgs& da, int C, const Epi& ep, float* partials, hipStream_t s) {
  constexpr int RPW = kWave / GL;
  constexpr int U = 4;
  const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * RPW);
  const int stg = epi_stage_kind(ep);
  const int nh = (int)n_heavy;
  if (stg == 1)
    flash_agg_kernel<GL, U, MAXH, 1><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep, partials);
  else if (stg == 2)
    flash_agg_kernel<GL, U, MAXH, 2><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep, partials);
  else
    flash_agg_kernel<GL, U, MAXH, 0><<<grid, kBlock, 0, s>>>(items, (int)n_items, heavy, nh, col, da, C, ep, partials);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

template <int GL>
static int launch_flash(const int4* items, int64_t n_items, int4* heavy, int64_t n_heavy, const int* col,
                        const DotArgs& da, int C, const Epi& ep, float* partials, hipStream_t s) {
  if (da.H <= 1) return launch_flash_h<GL, 1>(items, n_items, heavy, n_heavy, col, da, C, ep, partials, s);
  if (da.H <= 2) return launch_flash_h<GL, 2>(items, n_items, heavy, n_heavy, col, da, C, ep, partials, s);
  return launch_flash_h<GL, 4>(items, n_items, heavy, n_heavy, col, da, C, ep, partials, s);
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int64_t gnpde_attn_dot_partial_floats(int64_t heads, int64_t C) { return (heads * C + 2 * heads + 3) & ~(int64_t)3; }

int gnpde_attn_dot_supported(int64_t heads, int64_t dk, int64_t C) {
  const int64_t att = heads * dk;
  if (heads < 1 || heads > 4 || dk < 4 || dk % 4 || C < 1 || C > 256 || C % 4) return 0;
  const int64_t S = dk / 4;
  if (S & (S - 1)) return 0;
  // a 16-lane row holds att/4 distinct slices; att/4 must divide 16
  if (att > 64 || 16 % (att / 4)) return 0;
  return 1;
}

int gnpde_attn_dot_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                           const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads, int64_t dk,
                           int64_t C, const float* x, int64_t ldx, const float* x0, int64_t ldx0, const float* alpha,
                           const float* beta, int flags, float* f, int64_t ldf, float* partials, int64_t n_slots,
                           const gnpde_stage_epilogue_t* stage, void* stream) {
  GNPDE_REQUIRE(gnpde_attn_dot_supported(heads, dk, C), GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: heads=%lld dk=%lld C=%lld outside the fused kernel (heads <= 4, dk %% 4 == 0 with "
                "dk/4 a power of two, heads*dk <= 64 dividing 64, C %% 4 == 0, C <= 256)",
                (long long)heads, (long long)dk, (long long)C);
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf, stage);
  // the partial slots hold ps floats each (gnpde_attn_dot_partial_floats): check_epi
  // bounds n_slots * C, the wider slots are bounded here
  int rc = check_epi(ep, C, 0, partials, n_slots);
  if (rc) return rc;
  const int64_t ps = gnpde_attn_dot_partial_floats(heads, C);
  GNPDE_REQUIRE(n_heavy == 0 || (partials != nullptr && n_slots > 0), GNPDE_EINVAL,
                "attn_dot_rhs: hub rows need a partials buffer and its slot count");
  GNPDE_REQUIRE(n_slots >= 0 && n_slots * ps * 4 < (int64_t)kBufRecords, GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: %lld partial slots x %lld floats exceed the 4 GiB of 32-bit buffer offsets",
                (long long)n_slots, (long long)ps);
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0, GNPDE_EINVAL, "attn_dot_rhs: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && q && k), GNPDE_EINVAL, "attn_dot_rhs: NULL plan/col/q/k");
  GNPDE_REQUIRE(ldqk >= heads * dk && ldqk % 4 == 0 && aligned16(q) && aligned16(k), GNPDE_EUNSUPPORTED,
                "attn_dot_rhs: q/k rows must be 16-byte aligned (ldqk %% 4 == 0)");
  GNPDE_REQUIRE(ldx % 4 == 0 && ldf % 4 == 0 && aligned16(x) && (!f || aligned16(f)) && aligned16(partials),
                GNPDE_EUNSUPPORTED, "attn_dot_rhs: x / f rows must be 16-byte aligned");
  if (flags & GNPDE_ADD_SOURCE)
    GNPDE_REQUIRE(ldx0 % 4 == 0 && aligned16(x0), GNPDE_EUNSUPPORTED, "attn_dot_rhs: x0 rows must be 16-byte aligned");
  if (stage) {
    bool ok = !stage->f_out || aligned16(stage->f_out);
    for (int i = 0; i < stage->n_out; ++i) {
      ok = ok && aligned16(stage->o[i].out) && (!stage->o[i].base || aligned16(stage->o[i].base));
      for (int j = 0; j < stage->o[i].nk; ++j) ok = ok && aligned16(stage->o[i].k[j]);
    }
    GNPDE_REQUIRE(ok && (!stage->dot_rows || aligned16(stage->dot_with)), GNPDE_EUNSUPPORTED,
                  "attn_dot_rhs: stage rows must be 16-byte aligned");
  }
  if (n_items == 0) return GNPDE_OK;
  DotArgs da;
  da.q = q;
  da.k = k;
  da.ldqk = ldqk;
  da.H = (int)heads;
  da.S = (int)(dk / 4);
  da.qlanes = (int)(heads * dk / 4);
  da.scale = kLog2e / sqrtf((float)dk);
  da.ps = (int)ps;
  const int4* it = reinterpret_cast<const int4*>(items);
  int4* hv = reinterpret_cast<int4*>(heavy);
  const int lanes = (int)(C / 4);
  hipStream_t s = as_stream(stream);
  if (lanes <= 16) return launch_flash<16>(it, n_items, hv, n_heavy, col, da, (int)C, ep, partials, s);
  if (lanes <= 32) return launch_flash<32>(it, n_items, hv, n_heavy, col, da, (int)C, ep, partials, s);
  return launch_flash<64>(it, n_items, hv, n_heavy, col, da, (int)C, ep, partials, s);
}

}  // extern "C"
