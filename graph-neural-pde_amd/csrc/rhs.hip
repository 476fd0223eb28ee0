// rhs.hip — per-RHS-evaluation kernels: the Laplacian SpMM RHS (K1), the
// attention RHS (K3: softmax statistics + weighted aggregation) and the
// reference-mode key-sum node scores.
#include "aggregate.hpp"

namespace gnpde {

// ------------------------------------------------------------------ softmax statistics
// One wavefront per plan item over a grouped CSR (group g = the item's row).
// Lane per edge; per head an online (max, sum-exp) over 64-edge blocks.
template <int MAXH>
__global__ __launch_bounds__(256) void stats_kernel(const int4* __restrict__ items, int n_items,
                                                     const int* __restrict__ gidx, int group_is_dst, ScoreArgs sa,
                                                     double* __restrict__ m_out, float* __restrict__ rl_out,
                                                     double* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (wid >= n_items) return;
  const int4 it = items[wid];
  const int g = uniform(it.x), beg = uniform(it.y), end = uniform(it.z), slot = uniform(it.w);
  const int H = sa.H;
  double M[MAXH];
  float L[MAXH];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
  }
  for (int e0 = beg; e0 < end; e0 += kWave) {
    const int n = min(kWave, end - e0);
    const bool live = lane < n;
    const int o = live ? gidx[e0 + lane] : 0;
    const int src = group_is_dst ? o : g;
    const int dst = group_is_dst ? g : o;
#pragma unroll
    for (int h = 0; h < MAXH; ++h) {
      if (h < H) {
        const double s = live ? sa.score(src, dst, h) : -INFINITY;
        const double bm = wave_max(s);
        const double mn = fmax(M[h], bm);
        const float z = live ? expf((float)(s - mn)) : 0.f;
        const float bs = wave_sum(z);
        L[h] = (M[h] == -INFINITY ? 0.f : L[h] * expf((float)(M[h] - mn))) + bs;
        M[h] = mn;
      }
    }
  }
  if (lane != 0) return;
  for (int h = 0; h < H && h < MAXH; ++h) {
    if (slot >= 0) {
      partials[(int64_t)slot * 2 * H + h] = M[h];
      partials[(int64_t)slot * 2 * H + H + h] = (double)L[h];
    } else {
      m_out[(int64_t)g * H + h] = M[h];
      rl_out[(int64_t)g * H + h] = 1.0f / (L[h] + kSoftmaxEps);
    }
  }
}

// Hub groups: combine the chunks' (max, sum) pairs in plan order.
__global__ __launch_bounds__(256) void stats_fixup_kernel(const int4* __restrict__ heavy, int n_heavy, int H,
                                                           const double* __restrict__ partials,
                                                           double* __restrict__ m_out, float* __restrict__ rl_out) {
  const int t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_heavy * H) return;
  const int i = t / H, h = t - i * H;
  const int4 hv = heavy[i];
  const int g = hv.x, first = hv.y, nch = hv.z;
  double M = -INFINITY;
  for (int c = 0; c < nch; ++c) M = fmax(M, partials[(int64_t)(first + c) * 2 * H + h]);
  float L = 0.f;
  for (int c = 0; c < nch; ++c) {
    const double mc = partials[(int64_t)(first + c) * 2 * H + h];
    const float lc = (float)partials[(int64_t)(first + c) * 2 * H + H + h];
    if (mc != -INFINITY) L += lc * expf((float)(mc - M));
  }
  m_out[(int64_t)g * H + h] = M;
  rl_out[(int64_t)g * H + h] = 1.0f / (L + kSoftmaxEps);
}

// ------------------------------------------------------------------ per-edge attention (COO order)
__global__ __launch_bounds__(256) void edge_attention_kernel(const int4* __restrict__ items, int n_items,
                                                              const int* __restrict__ col,
                                                              const int* __restrict__ perm, int norm_idx,
                                                              ScoreArgs sa, const double* __restrict__ m,
                                                              const float* __restrict__ rl, float* __restrict__ att) {
  const int lane = threadIdx.x & 63;
  const int wid = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6));
  if (wid >= n_items) return;
  const int4 it = items[wid];
  const int row = uniform(it.x), beg = uniform(it.y), end = uniform(it.z);
  const int H = sa.H;
  for (int p = beg + lane; p < end; p += kWave) {
    const int c = col[p];
    const int g = norm_idx == 0 ? row : c;
    const int64_t e = perm[p];
    for (int h = 0; h < H; ++h) {
      const double s = sa.score(row, c, h);
      att[e * H + h] = expf((float)(s - m[(int64_t)g * H + h])) * rl[(int64_t)g * H + h];
    }
  }
}

// ------------------------------------------------------------------ reference-mode key sum
// partial column sums of indeg-weighted x over row tiles, fp64:
//   part[b][tile][c] = sum_{n in tile} indeg[b*N+n] * x[b*N+n][c];  part[..][C] = sum indeg
constexpr int kKeysumRows = 128;

__global__ __launch_bounds__(256) void keysum_partial_kernel(const float* __restrict__ x, int64_t N, int C,
                                                              int64_t ldx, const int* __restrict__ indeg,
                                                              int ntiles, double* __restrict__ part) {
  const int tile = blockIdx.x, b = blockIdx.y;
  const int64_t n0 = (int64_t)tile * kKeysumRows;
  const int64_t n1 = min<int64_t>(N, n0 + kKeysumRows);
  double* out = part + ((int64_t)b * ntiles + tile) * (C + 1);
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    double s = 0.0;
    for (int64_t n = n0; n < n1; ++n) {
      const int64_t r = (int64_t)b * N + n;
      const double d = (double)indeg[r];
      s += (c < C) ? d * (double)x[r * ldx + c] : d;
    }
    out[c] = s;
  }
}

// per batch element: Xbar, S = Wk Xbar + E bk, U[c,h] = sum_{d in h} Wq[d,c] S[d] / sqrt(dk), v[h]
__global__ __launch_bounds__(256) void keysum_finish_kernel(const double* __restrict__ part, int ntiles, int C,
                                                             const float* __restrict__ Wq,
                                                             const float* __restrict__ bq,
                                                             const float* __restrict__ Wk,
                                                             const float* __restrict__ bk, int att, int H,
                                                             double* __restrict__ U, double* __restrict__ v) {
  extern __shared__ __attribute__((aligned(16))) double sm[];
  double* xbar = sm;             // C+1
  double* S = sm + (C + 1);      // att
  const int b = blockIdx.x;
  const double* pb = part + (int64_t)b * ntiles * (C + 1);
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    double s = 0.0;
    for (int t = 0; t < ntiles; ++t) s += pb[(int64_t)t * (C + 1) + c];
    xbar[c] = s;
  }
  __syncthreads();
  const double esum = xbar[C];
  for (int d = threadIdx.x; d < att; d += blockDim.x) {
    double s = esum * (double)bk[d];
    for (int c = 0; c < C; ++c) s += (double)Wk[(int64_t)d * C + c] * xbar[c];
    S[d] = s;
  }
  __syncthreads();
  const int dk = att / H;
  const double inv = 1.0 / sqrt((double)dk);
  for (int t = threadIdx.x; t < C * H; t += blockDim.x) {
    const int c = t / H, h = t - c * H;
    double s = 0.0;
    for (int d = h * dk; d < (h + 1) * dk; ++d) s += (double)Wq[(int64_t)d * C + c] * S[d];
    U[((int64_t)b * C + c) * H + h] = s * inv;
  }
  for (int h = threadIdx.x; h < H; h += blockDim.x) {
    double s = 0.0;
    for (int d = h * dk; d < (h + 1) * dk; ++d) s += (double)bq[d] * S[d];
    v[(int64_t)b * H + h] = s * inv;
  }
}

// cs[r,h] = x_r . U[b,:,h] + v[b,h]  (fp64), one wavefront per row
template <int MAXH>
__global__ __launch_bounds__(256) void node_scores_kernel(const float* __restrict__ x, int64_t R, int64_t N, int C,
                                                           int64_t ldx, int H, const double* __restrict__ U,
                                                           const double* __restrict__ v, double* __restrict__ cs) {
  const int lane = threadIdx.x & 63;
  const int64_t nw = (int64_t)gridDim.x * kWavesPerBlock;
  for (int64_t r = uniform(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); r < R; r += nw) {
    const int64_t b = r / N;
    double acc[MAXH];
#pragma unroll
    for (int h = 0; h < MAXH; ++h) acc[h] = 0.0;
    for (int c = lane; c < C; c += kWave) {
      const double xv = (double)x[r * ldx + c];
      const double* u = U + (b * C + c) * H;
#pragma unroll
      for (int h = 0; h < MAXH; ++h)
        if (h < H) acc[h] = fma(xv, u[h], acc[h]);
    }
#pragma unroll
    for (int h = 0; h < MAXH; ++h) {
      if (h < H) {
        const double s = wave_sum(acc[h]);
        if (lane == 0) cs[r * H + h] = s + v[b * H + h];
      }
    }
  }
}

static int check_score_args(int mode, int64_t heads, int64_t dk, const double* cs, const float* q, const float* k) {
  GNPDE_REQUIRE(heads >= 1 && heads <= 16, GNPDE_EUNSUPPORTED, "attention: heads=%lld not in [1,16]",
                (long long)heads);
  GNPDE_REQUIRE(mode >= GNPDE_SCORE_REFERENCE && mode <= GNPDE_SCORE_PEARSON, GNPDE_EINVAL,
                "attention: unknown score mode %d", mode);
  if (mode == GNPDE_SCORE_REFERENCE) {
    GNPDE_REQUIRE(cs != nullptr, GNPDE_EINVAL, "attention: reference mode needs cs");
  } else {
    GNPDE_REQUIRE(q != nullptr && k != nullptr && dk >= 1, GNPDE_EINVAL, "attention: per-edge mode needs q, k, dk");
  }
  return GNPDE_OK;
}

static ScoreArgs make_score_args(int mode, int64_t heads, int64_t dk, const double* cs, const float* q,
                                 const float* k, int64_t ldqk, float p0, float p1) {
  ScoreArgs sa;
  sa.mode = mode;
  sa.H = (int)heads;
  sa.dk = (int)dk;
  sa.cs = cs;
  sa.q = q;
  sa.k = k;
  sa.ldqk = ldqk;
  sa.p0 = p0;
  sa.p1 = p1;
  return sa;
}

static Epi make_epi(const float* x, int64_t ldx, const float* x0, int64_t ldx0, const float* alpha, const float* beta,
                    int flags, float* f, int64_t ldf) {
  Epi e;
  e.x = x;
  e.ldx = ldx;
  e.x0 = x0;
  e.ldx0 = ldx0;
  e.alpha = alpha;
  e.beta = beta;
  e.flags = flags;
  e.f = f;
  e.ldf = ldf;
  return e;
}

static int check_epi(const Epi& e, int64_t C, int64_t n_heavy, const void* partials) {
  GNPDE_REQUIRE(C >= 1, GNPDE_EINVAL, "rhs: C must be >= 1");
  GNPDE_REQUIRE(e.x && e.f, GNPDE_EINVAL, "rhs: NULL x or f");
  GNPDE_REQUIRE(e.ldx >= C && e.ldf >= C, GNPDE_EINVAL, "rhs: leading dimension < C");
  if (e.flags & GNPDE_EPI_RHS) GNPDE_REQUIRE(e.alpha != nullptr, GNPDE_EINVAL, "rhs: NULL alpha");
  if (e.flags & GNPDE_ADD_SOURCE) {
    GNPDE_REQUIRE(e.flags & GNPDE_EPI_RHS, GNPDE_EINVAL, "rhs: ADD_SOURCE needs EPI_RHS");
    GNPDE_REQUIRE(e.x0 && e.beta && e.ldx0 >= C, GNPDE_EINVAL, "rhs: ADD_SOURCE needs x0, beta, ldx0 >= C");
  }
  GNPDE_REQUIRE(n_heavy == 0 || partials != nullptr, GNPDE_EINVAL, "rhs: hub rows need a partials buffer");
  return GNPDE_OK;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_spmm_rhs_f32(const int32_t* items, int64_t n_items, const int32_t* heavy, int64_t n_heavy,
                       const int32_t* col, const float* w, int64_t C, const float* x, int64_t ldx, const float* x0,
                       int64_t ldx0, const float* alpha, const float* beta, int flags, float* f, int64_t ldf,
                       float* partials, void* stream) {
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf);
  int rc = check_epi(ep, C, n_heavy, partials);
  if (rc) return rc;
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0, GNPDE_EINVAL, "spmm_rhs: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && w), GNPDE_EINVAL, "spmm_rhs: NULL plan/col/w");
  PlainWeights wp{w};
  return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
}

int gnpde_softmax_stats_f32(const int32_t* items, int64_t n_items, const int32_t* heavy, int64_t n_heavy,
                            const int32_t* gidx, int group_is_dst, int mode, int64_t heads, int64_t dk,
                            const double* cs, const float* q, const float* k, int64_t ldqk, float score_p0,
                            float score_p1, double* m, float* rl, double* partials, void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE(m && rl, GNPDE_EINVAL, "softmax_stats: NULL m/rl");
  GNPDE_REQUIRE(n_heavy == 0 || partials, GNPDE_EINVAL, "softmax_stats: hub groups need partials");
  if (n_items == 0) return GNPDE_OK;
  GNPDE_REQUIRE(items && gidx, GNPDE_EINVAL, "softmax_stats: NULL items/gidx");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  hipStream_t s = as_stream(stream);
  const int4* it = reinterpret_cast<const int4*>(items);
  const unsigned grid = (unsigned)ceil_div(n_items, kWavesPerBlock);
  if (heads <= 1)
    stats_kernel<1><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, m, rl, partials);
  else if (heads <= 2)
    stats_kernel<2><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, m, rl, partials);
  else if (heads <= 4)
    stats_kernel<4><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, m, rl, partials);
  else if (heads <= 8)
    stats_kernel<8><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, m, rl, partials);
  else
    stats_kernel<16><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, m, rl, partials);
  GNPDE_LAUNCH_CHECK();
  if (n_heavy > 0) {
    const unsigned g2 = (unsigned)ceil_div(n_heavy * heads, kBlock);
    stats_fixup_kernel<<<g2, kBlock, 0, s>>>(reinterpret_cast<const int4*>(heavy), (int)n_heavy, (int)heads, partials,
                                             m, rl);
    GNPDE_LAUNCH_CHECK();
  }
  return GNPDE_OK;
}

int gnpde_attn_rhs_f32(const int32_t* items, int64_t n_items, const int32_t* heavy, int64_t n_heavy,
                       const int32_t* col, int norm_idx, int mode, int64_t heads, int64_t dk, const double* cs,
                       const float* q, const float* k, int64_t ldqk, float score_p0, float score_p1, const double* m,
                       const float* rl, int64_t C, const float* x, int64_t ldx, const float* x0, int64_t ldx0,
                       const float* alpha, const float* beta, int flags, float* f, int64_t ldf, float* partials,
                       void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf);
  rc = check_epi(ep, C, n_heavy, partials);
  if (rc) return rc;
  GNPDE_REQUIRE(norm_idx == 0 || norm_idx == 1, GNPDE_EINVAL, "attn_rhs: norm_idx must be 0 or 1");
  GNPDE_REQUIRE(m && rl, GNPDE_EINVAL, "attn_rhs: NULL m/rl");
  GNPDE_REQUIRE(n_items == 0 || (items && col), GNPDE_EINVAL, "attn_rhs: NULL plan/col");
  AttnWeights wp;
  wp.sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  wp.norm_idx = norm_idx;
  wp.m = m;
  wp.rl = rl;
  wp.invH = 1.0f / (float)heads;
  return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
}

int gnpde_edge_attention_f32(const int32_t* items, int64_t n_items, const int32_t* col, const int32_t* perm,
                             int norm_idx, int mode, int64_t heads, int64_t dk, const double* cs, const float* q,
                             const float* k, int64_t ldqk, float score_p0, float score_p1, const double* m,
                             const float* rl, float* att, void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE(norm_idx == 0 || norm_idx == 1, GNPDE_EINVAL, "edge_attention: norm_idx must be 0 or 1");
  if (n_items == 0) return GNPDE_OK;
  GNPDE_REQUIRE(items && col && perm && m && rl && att, GNPDE_EINVAL, "edge_attention: NULL pointer");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  const unsigned grid = (unsigned)ceil_div(n_items, kWavesPerBlock);
  edge_attention_kernel<<<grid, kBlock, 0, as_stream(stream)>>>(reinterpret_cast<const int4*>(items), (int)n_items,
                                                                col, perm, norm_idx, sa, m, rl, att);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

size_t gnpde_keysum_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t att) {
  (void)att;
  const int64_t ntiles = ceil_div(N, kKeysumRows);
  const int64_t H = 16;  // upper bound on heads
  return sizeof(double) * (size_t)(B * ntiles * (C + 1) + B * C * H + B * H) + 256;
}

int gnpde_ref_scores_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                         const float* Wq, const float* bq, const float* Wk, const float* bk, int64_t att,
                         int64_t heads, double* cs, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(x && indeg && Wq && bq && Wk && bk && cs && workspace, GNPDE_EINVAL, "ref_scores: NULL pointer");
  GNPDE_REQUIRE(B >= 1 && N >= 1 && C >= 1 && ldx >= C, GNPDE_EINVAL, "ref_scores: bad sizes");
  GNPDE_REQUIRE(heads >= 1 && heads <= 16 && att % heads == 0, GNPDE_EUNSUPPORTED,
                "ref_scores: heads must divide attention_dim and be <= 16");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_keysum_workspace_bytes(B, N, C, att), GNPDE_EINVAL,
                "ref_scores: workspace too small");
  GNPDE_REQUIRE(C + 1 + att <= 6000, GNPDE_EUNSUPPORTED, "ref_scores: C + attention_dim too large");
  hipStream_t s = as_stream(stream);
  const int ntiles = (int)ceil_div(N, kKeysumRows);
  double* part = static_cast<double*>(workspace);
  double* U = part + B * ntiles * (C + 1);
  double* v = U + B * C * heads;
  keysum_partial_kernel<<<dim3(ntiles, (unsigned)B), kBlock, 0, s>>>(x, N, (int)C, ldx, indeg, ntiles, part);
  GNPDE_LAUNCH_CHECK();
  const size_t shm = sizeof(double) * (size_t)(C + 1 + att);
  keysum_finish_kernel<<<(unsigned)B, kBlock, shm, s>>>(part, ntiles, (int)C, Wq, bq, Wk, bk, (int)att, (int)heads,
                                                        U, v);
  GNPDE_LAUNCH_CHECK();
  const int64_t R = B * N;
  const unsigned grid = (unsigned)std::min<int64_t>(ceil_div(R, kWavesPerBlock), 8192);
  if (heads <= 1)
    node_scores_kernel<1><<<grid, kBlock, 0, s>>>(x, R, N, (int)C, ldx, (int)heads, U, v, cs);
  else if (heads <= 2)
    node_scores_kernel<2><<<grid, kBlock, 0, s>>>(x, R, N, (int)C, ldx, (int)heads, U, v, cs);
  else if (heads <= 4)
    node_scores_kernel<4><<<grid, kBlock, 0, s>>>(x, R, N, (int)C, ldx, (int)heads, U, v, cs);
  else if (heads <= 8)
    node_scores_kernel<8><<<grid, kBlock, 0, s>>>(x, R, N, (int)C, ldx, (int)heads, U, v, cs);
  else
    node_scores_kernel<16><<<grid, kBlock, 0, s>>>(x, R, N, (int)C, ldx, (int)heads, U, v, cs);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
