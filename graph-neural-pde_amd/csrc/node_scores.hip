// node_scores.hip — the per-RHS score and softmax pieces of the attention RHS
// around K1 (kept out of rhs.hip so that they rebuild without K1's
// instantiations): softmax statistics over grouped CSRs and their hub fixup,
// edge-parallel head-mean weights and per-edge attention, the team-mode
// (per-edge q/k) kernels, and the reference-mode node scores (indegree-weighted
// key sum + node scores, gnpde_ref_scores_f32).
// Reference: SpGraphTransAttentionLayer.forward, src/function_transformer_attention.py:218-266;
// utils.softmax, src/utils.py:116-127.
#include "aggregate.hpp"
#include "rhs_host.hpp"

namespace gnpde {

// ------------------------------------------------------------------ softmax statistics
// GL lanes per plan item (64/GL items per wavefront).  Every lane keeps an
// online (max, sum-exp) per head over its strided edges; the GL partial states
// are merged by a fixed xor tree (deterministic).
template <int MAXH, int GL>
__global__ __launch_bounds__(256) void stats_kernel(const int4* __restrict__ items, int n_items,
                                                     const int* __restrict__ gidx, int group_is_dst, ScoreArgs sa,
                                                     double* __restrict__ m_out, float* __restrict__ rl_out,
                                                     float* __restrict__ mr_out, double* __restrict__ partials) {
  constexpr int G = kWave / GL;
  const int lane = threadIdx.x & 63;
  const int g = lane / GL, gl = lane % GL;
  const int item = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * G + g;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int grp = it.x, beg = it.y, end = it.z, slot = it.w;
  const int H = sa.H;
  double M[MAXH];
  float L[MAXH];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
  }
  for (int p = beg + gl; p < end; p += GL) {
    const int o = gidx[p];
    const int src = group_is_dst ? o : grp;
    const int dst = group_is_dst ? grp : o;
#pragma unroll
    for (int h = 0; h < MAXH; ++h)
      if (h < H) online_push(M[h], L[h], sa.score(src, dst, h));
  }
#pragma unroll
  for (int o = 1; o < GL; o <<= 1) {
#pragma unroll
    for (int h = 0; h < MAXH; ++h) {
      const double M2 = __shfl_xor(M[h], o);
      const float L2 = __shfl_xor(L[h], o);
      online_merge(M[h], L[h], M2, L2);
    }
  }
  if (!live || gl != 0) return;
  for (int h = 0; h < H && h < MAXH; ++h) {
    if (slot >= 0) {
      partials[(int64_t)slot * 2 * H + h] = M[h];
      partials[(int64_t)slot * 2 * H + H + h] = (double)L[h];
    } else {
      store_stats(m_out, rl_out, mr_out, grp, H, h, M[h], L[h]);
    }
  }
}

// Hub groups: one wavefront per (group, head) merging that group's chunk
// statistics (stats_merge_store, scores.hpp).
__global__ __launch_bounds__(256) void stats_fixup_kernel(const int4* __restrict__ heavy, int n_heavy, int H,
                                                           const double* __restrict__ partials,
                                                           double* __restrict__ m_out, float* __restrict__ rl_out,
                                                           float* __restrict__ mr_out) {
  const int wid = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (wid >= n_heavy * H) return;
  const int i = wid / H, h = wid - i * H;
  const int4 hv = heavy[i];
  stats_merge_store(hv.x, hv.y, hv.z, H, h, partials, m_out, rl_out, mr_out);
}

int launch_stats_fixup(const int4* heavy, int64_t n_heavy, int H, const double* partials, double* m, float* rl,
                       float* mr, hipStream_t s) {
  if (n_heavy <= 0) return GNPDE_OK;
  const unsigned g2 = (unsigned)ceil_div(n_heavy * H, kWavesPerBlock);
  stats_fixup_kernel<<<g2, kBlock, 0, s>>>(heavy, (int)n_heavy, H, partials, m, rl, mr);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

// ------------------------------------------------------------------ edge-parallel weights
// w[p] = (sum_h exp(s_p,h - m[g,h]) * rl[g,h]) / H   (softmax, then mean over heads)
__global__ __launch_bounds__(256) void attn_weights_kernel(const int* __restrict__ rowidx, const int* __restrict__ col,
                                                            int64_t nnz, int norm_idx, ScoreArgs sa,
                                                            const double* __restrict__ m,
                                                            const float* __restrict__ rl, float* __restrict__ w) {
  const int H = sa.H;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
    const int r = rowidx[p], c = col[p];
    const int64_t g = norm_idx == 0 ? r : c;
    float acc = 0.f;
    for (int h = 0; h < H; ++h) {
      const double s = sa.score(r, c, h);
      acc += expf((float)(s - m[g * H + h])) * rl[g * H + h];
    }
    w[p] = acc / (float)H;
  }
}

// att[perm[p]*H + h] = exp(s_p,h - m[g,h]) * rl[g,h]   (COO order, per head)
__global__ __launch_bounds__(256) void edge_attention_kernel(const int* __restrict__ rowidx,
                                                              const int* __restrict__ col,
                                                              const int* __restrict__ perm, int64_t nnz,
                                                              int norm_idx, ScoreArgs sa,
                                                              const double* __restrict__ m,
                                                              const float* __restrict__ rl, float* __restrict__ att) {
  const int H = sa.H;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
    const int r = rowidx[p], c = col[p];
    const int64_t g = norm_idx == 0 ? r : c;
    const int64_t e = perm[p];
    for (int h = 0; h < H; ++h) {
      const double s = sa.score(r, c, h);
      att[e * H + h] = expf((float)(s - m[g * H + h])) * rl[g * H + h];
    }
  }
}

// ------------------------------------------------------------------ team-mode kernels (per-edge q/k scores)
// Team-mode softmax statistics: one team of T lanes per work item.  The
// item's own row (q of the source group, or k of the destination group) is
// loaded once; the other endpoints' indices come in T at a time (one per
// lane, then broadcast with shuffles) and kTeamEdges rows are in flight
// together.  Edges are pushed in CSR order, as the lane-mode kernel does.
// Loop trip counts are wave-uniform (maxima over the wave's teams), so every
// shuffle runs with the whole wavefront active; a team past its own edges
// computes throw-away scores and pushes nothing.
constexpr int kTeamEdges = 4;

template <int VEC>
__global__ __launch_bounds__(256) void stats_team_kernel(const int4* __restrict__ items, int n_items,
                                                          const int* __restrict__ gidx, int group_is_dst, ScoreArgs sa,
                                                          Team tm, double* __restrict__ m_out,
                                                          float* __restrict__ rl_out, float* __restrict__ mr_out,
                                                          double* __restrict__ partials) {
  const int lane = threadIdx.x & 63;
  const int T = tm.T, S = tm.S, tpw = kWave / T;
  const int team = lane / T, t = lane % T, h = t / S;
  const int item = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * tpw + team;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, -1);
  const int grp = it.x, beg = it.y, end = it.z, slot = it.w;
  float own[VEC];
  team_row<VEC>(sa, group_is_dst ? sa.k : sa.q, grp, t, own);
  const float* __restrict__ other_base = group_is_dst ? sa.q : sa.k;
  double M = -INFINITY;
  float L = 0.f;
  const int rounds = wave_max_int((end - beg + T - 1) / T);
  for (int r = 0; r < rounds; ++r) {
    const int p0 = beg + r * T;
    const int cnt = max(0, min(T, end - p0));
    int mine = 0;
    if (cnt > 0) mine = gidx[p0 + min(t, cnt - 1)];
    const int jmax = wave_max_int(cnt);
    for (int j = 0; j < jmax; j += kTeamEdges) {
      float other[kTeamEdges][VEC];
#pragma unroll
      for (int u = 0; u < kTeamEdges; ++u) {
        const int o = __shfl(mine, team * T + max(0, min(j + u, cnt - 1)));
        team_row<VEC>(sa, other_base, o, t, other[u]);
      }
      float s[kTeamEdges];
#pragma unroll
      for (int u = 0; u < kTeamEdges; ++u)
        s[u] = group_is_dst ? team_score_regs<VEC>(sa, other[u], own, S) : team_score_regs<VEC>(sa, own, other[u], S);
#pragma unroll
      for (int u = 0; u < kTeamEdges; ++u)
        if (j + u < cnt) online_push(M, L, (double)s[u]);
    }
  }
  if (!live || (t % S) != 0) return;
  const int H = sa.H;
  if (slot >= 0) {
    partials[(int64_t)slot * 2 * H + h] = M;
    partials[(int64_t)slot * 2 * H + H + h] = (double)L;
  } else {
    store_stats(m_out, rl_out, mr_out, grp, H, h, M, L);
  }
}

// Team-mode attention weights: a team takes T consecutive edges (indices
// loaded one per lane, coalesced), then evaluates them kTeamEdges at a time
// with the q/k rows and the group's softmax statistics all in flight.  Trip
// counts are wave-uniform, as in stats_team_kernel.
template <int VEC, bool COO>
__global__ __launch_bounds__(256) void attn_team_kernel(const int* __restrict__ rowidx, const int* __restrict__ col,
                                                         const int* __restrict__ perm, int64_t nnz, int norm_idx,
                                                         ScoreArgs sa, Team tm, const double* __restrict__ m,
                                                         const float* __restrict__ rl, float* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int T = tm.T, S = tm.S, tpw = kWave / T;
  const int team = lane / T, t = lane % T, h = t / S;
  const int H = sa.H;
  const bool leader = (t % S) == 0;
  const __amdgpu_buffer_rsrc_t rout = buf_rsrc(out);
  const int64_t wave_first = (int64_t)(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * tpw * T;
  const int64_t sweep = (int64_t)gridDim.x * kWavesPerBlock * tpw * T;
  for (int64_t w0 = wave_first; w0 < nnz; w0 += sweep) {
    const int64_t p0 = w0 + (int64_t)team * T;
    const int cnt = (int)max((int64_t)0, min((int64_t)T, nnz - p0));
    int my_r = 0, my_c = 0, my_dst = 0;
    if (cnt > 0) {
      const int64_t pm = p0 + min(t, cnt - 1);
      my_r = rowidx[pm];
      my_c = col[pm];
      if (COO) my_dst = perm[pm];
    }
    const int jmax = wave_max_int(cnt);
    for (int j = 0; j < jmax; j += kTeamEdges) {
      float qv[kTeamEdges][VEC], kv[kTeamEdges][VEC];
      double mv[kTeamEdges];
      float rv[kTeamEdges];
      int dst[kTeamEdges];
#pragma unroll
      for (int u = 0; u < kTeamEdges; ++u) {
        const int src = team * T + max(0, min(j + u, cnt - 1));
        const int r = __shfl(my_r, src), c = __shfl(my_c, src);
        dst[u] = COO ? __shfl(my_dst, src) : 0;
        team_row<VEC>(sa, sa.q, r, t, qv[u]);
        team_row<VEC>(sa, sa.k, c, t, kv[u]);
        const int64_t g = norm_idx == 0 ? r : c;
        mv[u] = m[g * H + h];
        rv[u] = rl[g * H + h];
      }
#pragma unroll
      for (int u = 0; u < kTeamEdges; ++u) {
        const float s = team_score_regs<VEC>(sa, qv[u], kv[u], S);
        float term = leader ? expf((float)((double)s - mv[u])) * rv[u] : 0.f;
        if (COO) {
          const bool st = leader && j + u < cnt;
          buf_store_f32(rout, st ? (uint32_t)(((int64_t)dst[u] * H + h) * 4) : kBufNone, term);
        } else {
          for (int o = S; o < T; o <<= 1) term += __shfl_xor(term, o);
          const bool st = t == 0 && j + u < cnt;
          buf_store_f32(rout, st ? (uint32_t)((p0 + j + u) * 4) : kBufNone, term / (float)H);
        }
      }
    }
  }
}

// ------------------------------------------------------------------ reference-mode key sum
// The fork's global key sum S = sum_e k_dst(e) = Wk xbar + E bk with
// xbar = sum_n indeg(n) x_n is linear in the rows, so every row tile carries
// its own share of S.  Three launches, no tickets:
//   keysum_partial: per tile, xt = sum_{n in tile} indeg(n) x[b,n,:] (fp64,
//                   xt[C] = sum indeg), then St = Wk xt + xt[C] bk  -> part[b][tile][att]
//                   (about 256 tiles per launch);
//   key_projection: one 1024-thread workgroup per batch element sums the tile
//                   shares of S (fixed order), forms U = Wq^T S / sqrt(dk) and v;
//   node_scores:    cs = x . U + v with U[b] loaded from the workspace.
// KS_BLOCK threads per tile, TPR threads per row, RPB = KS_BLOCK/TPR rows in
// flight per iteration (16-byte loads, 8 rows unrolled per thread).
constexpr int kKeysumBlock = 1024;
#ifndef GNPDE_KS_ROWS
#define GNPDE_KS_ROWS 4  // 4 / 8 / 12: 0.1423 / 0.1429 / 0.1437 ms per reference RHS (with ring depth 2 / 4 / 6)
#endif
constexpr int kKeysumRows = GNPDE_KS_ROWS;  // rows per thread in flight (keysum_partial)
constexpr int kKeysumTilesTarget = 256;  // tiles per launch: the projection block reads them all
constexpr int kProjLanes = 32;           // lanes per row of Wk (S phase)
constexpr int kProjLoads = 16;           // tile shares in flight per thread (key_projection)

template <int VEC>
__global__ __launch_bounds__(kKeysumBlock) void keysum_partial_kernel(const float* __restrict__ x, int64_t N, int C,
                                                                       int64_t ldx, const int* __restrict__ indeg,
                                                                       const float* __restrict__ Wk,
                                                                       const float* __restrict__ bk, int att,
                                                                       int rows_per_tile, int TPR, int ntiles,
                                                                       double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double red[];  // [RPB][C+1] | xt[C+1]
  const int tile = blockIdx.x, b = blockIdx.y;
  const int RPB = blockDim.x / TPR;
  const int rs = threadIdx.x / TPR, t = threadIdx.x % TPR;
  const int64_t n0 = (int64_t)tile * rows_per_tile;
  const int64_t n1 = min<int64_t>(N, n0 + rows_per_tile);
  const int64_t base = (int64_t)b * N;
  for (int c0 = t * VEC; c0 < C; c0 += TPR * VEC) {
    double acc[VEC];
#pragma unroll
    for (int i = 0; i < VEC; ++i) acc[i] = 0.0;
    // KSB rows per thread in flight: every load of a batch issued before its sums (the
    // loop was one memory latency per 4 rows, ~5 in a row per thread: 18.4 us on G-arxiv)
    for (int64_t nb = n0 + rs; nb < n1; nb += (int64_t)RPB * kKeysumRows) {
      float v[kKeysumRows][VEC];
      int dg[kKeysumRows];
#pragma unroll
      for (int k = 0; k < kKeysumRows; ++k) {
        const int64_t n = nb + (int64_t)k * RPB;
        const int64_t nn = n < n1 ? n : n0;  // past the tile: a row of it again, weighted 0
        load_vec<VEC>(x + (base + nn) * ldx + c0, v[k]);
        dg[k] = n < n1 ? indeg[base + nn] : 0;
      }
#pragma unroll
      for (int k = 0; k < kKeysumRows; ++k) {
        if (nb + (int64_t)k * RPB < n1) {  // same sums, same order as one row at a time
          const double d = (double)dg[k];
#pragma unroll
          for (int i = 0; i < VEC; ++i) acc[i] = fma(d, (double)v[k][i], acc[i]);
        }
      }
    }
#pragma unroll
    for (int i = 0; i < VEC; ++i) red[rs * (C + 1) + c0 + i] = acc[i];
  }
  if (t == 0) {
    double ds = 0.0;
    for (int64_t n = n0 + rs; n < n1; n += RPB) ds += (double)indeg[base + n];
    red[rs * (C + 1) + C] = ds;
  }
  __syncthreads();
  double* xt = red + RPB * (C + 1);
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    double sum = 0.0;
    for (int r = 0; r < RPB; ++r) sum += red[r * (C + 1) + c];  // row-slot order: deterministic
    xt[c] = sum;
  }
  __syncthreads();
  // this tile's share of S: kProjLanes lanes per row of Wk, xor tree over them
  const int l = threadIdx.x % kProjLanes;
  double* __restrict__ pb = part + ((int64_t)b * ntiles + tile) * att;
  for (int d0 = 0; d0 < att; d0 += kKeysumBlock / kProjLanes) {
    const int d = d0 + threadIdx.x / kProjLanes;
    const int dd = min(d, att - 1);
    double acc = 0.0;
#pragma unroll 4
    for (int c = l; c < C; c += kProjLanes) acc = fma((double)Wk[(int64_t)dd * C + c], xt[c], acc);
#pragma unroll
    for (int o = kProjLanes / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
    if (l == 0 && d < att) pb[d] = acc + xt[C] * (double)bk[d];
  }
}

// Per batch element b (one workgroup of kKeysumBlock threads), from the tile
// shares:  S = sum_tiles St  (the fork's global key sum, :249),
//   U[c,h] = sum_{d in head h} Wq[d,c] S[d] / sqrt(dk)   (padded [Cp][Hp], zeros past C, H)
//   v[h]   = bq_h . S_h / sqrt(dk)                       (stored as row c = Cp of U)
// so that cs[n,h] = x_n . U[:,h] + v[h] = q_{n,h} . S_h / sqrt(dk).  U, v go to
// the workspace (uv[b] = U[Cp*Hp] | v[Hp]).  The launch is latency-bound, so
// every global load is issued at the start: the tile shares (kProjLoads per
// thread) and the thread's slice of Wq / bq (kProjW values: thread (j, h, c)
// takes rows d = h*dk + j, + J, ... of its head, J splits per output).  Sums run
// in a fixed order (tiles, then tile groups; rows, then splits).
constexpr int kProjW = 8;  // Wq values prefetched per thread

__global__ __launch_bounds__(kKeysumBlock) void key_projection_kernel(const double* __restrict__ part, int ntiles,
                                                                       int C, const float* __restrict__ Wq,
                                                                       const float* __restrict__ bq, int att, int H,
                                                                       int Cp, int Hp, double* __restrict__ uv) {
  extern __shared__ __attribute__((aligned(16))) double kp_lds[];  // S[att] | red[kKeysumBlock]
  double* S = kp_lds;
  double* red = S + att;
  const int b = blockIdx.x;
  const int tid = threadIdx.x;
  const int dk = att / H;
  const double inv = 1.0 / sqrt((double)dk);
  double* __restrict__ U = uv + (int64_t)b * (Cp * Hp + Hp);
  // output pairs (h, c), c = Cp being v; J splits of the head's rows per pair
  const int P = (Cp + 1) * Hp;
  const int J = P <= kKeysumBlock ? max(1, min(kKeysumBlock / P, dk)) : 1;
  const bool pre = P <= kKeysumBlock && (dk + J - 1) / J <= kProjW;
  const int pj = tid / P, pq = tid - pj * P;
  const int ph = pq / (Cp + 1), pc = pq - ph * (Cp + 1);
  float wq[kProjW];
  if (pre) {
#pragma unroll
    for (int i = 0; i < kProjW; ++i) {
      const int dd = pj + J * i;
      const bool ok = pj < J && ph < H && dd < dk && (pc < C || pc == Cp);
      const int d = ph * dk + (ok ? dd : 0);
      wq[i] = ok ? (pc == Cp ? bq[d] : Wq[(int64_t)d * C + pc]) : 0.f;
    }
  }
  const double* __restrict__ pb = part + (int64_t)b * ntiles * att;
  // S: rows of att in chunks of DW, TG tile groups per chunk; thread (tg, d) sums
  // tiles tg, tg + TG, ... in tile order, then the TG group sums in group order
  const int DW = min(att, kKeysumBlock), TG = kKeysumBlock / DW;
  const int tg = tid / DW, dl = tid - tg * DW;
  for (int d0 = 0; d0 < att; d0 += DW) {
    const int d = d0 + dl;
    double acc = 0.0;
    if (tg < TG && d < att) {
      for (int t0 = tg; t0 < ntiles; t0 += kProjLoads * TG) {
        double v[kProjLoads];
#pragma unroll
        for (int k = 0; k < kProjLoads; ++k) v[k] = pb[(int64_t)min(t0 + k * TG, ntiles - 1) * att + d];
#pragma unroll
        for (int k = 0; k < kProjLoads; ++k)
          if (t0 + k * TG < ntiles) acc += v[k];
      }
    }
    red[tid] = acc;
    __syncthreads();
    if (tid < DW && d0 + tid < att) {
      double sum = 0.0;
      for (int g = 0; g < TG; ++g) sum += red[g * DW + tid];
      S[d0 + tid] = sum;
    }
    __syncthreads();
  }
  if (pre) {
    double a = 0.0;
#pragma unroll
    for (int i = 0; i < kProjW; ++i) {
      const int dd = pj + J * i;
      if (pj < J && ph < H && dd < dk) a = fma((double)wq[i], S[ph * dk + dd], a);
    }
    red[tid] = a;
    __syncthreads();
    if (tid < P) {
      double sum = 0.0;
      for (int j = 0; j < J; ++j) sum += red[j * P + tid];
      U[pc * Hp + ph] = sum * inv;
    }
    return;
  }
  // general shapes: one thread per output, Wq / bq loaded in the loop
  for (int t = tid; t < P; t += blockDim.x) {
    const int h = t / (Cp + 1), c = t - h * (Cp + 1);
    double a = 0.0;
    if (h < H && (c < C || c == Cp)) {
#pragma unroll 16
      for (int d = h * dk; d < (h + 1) * dk; ++d)
        a = fma((double)(c == Cp ? bq[d] : Wq[(int64_t)d * C + c]), S[d], a);
    }
    U[c * Hp + h] = a * inv;
  }
}

// cs[b*N+n, h] = x_{b,n} . U[b,:,h] + v[b,h]  (fp64 accumulation).
// GL lanes per row, G = 64/GL rows per wavefront step; each lane owns NPV
// columns of a chunk of CW = GL*NPV columns.  When the row fits one chunk (the
// usual case) the lane's slice of U[b] stays in registers for every row the
// wave visits and the next row's x slice is prefetched while the current one
// is reduced.  U is padded ([Cp][Hp], Cp = nch*CW, Hp = MAXH), so its loads
// take compile-time offsets from one lane base; x loads past C (ragged last
// chunk only) are clamped and zeroed.  No load sits behind a branch.
constexpr int kNodeScoreURegs = 32;  // doubles of U held per lane

template <int MAXH>
constexpr int node_scores_npv() { return kNodeScoreURegs / MAXH; }

template <int VEC, int NP, int GL, bool CLAMP>
__device__ __forceinline__ void ns_load_x(const float* __restrict__ xrow, int cbase, int gl, int C,
                                          float (&xv)[NP][VEC]) {
#pragma unroll
  for (int p = 0; p < NP; ++p) {
    const int c0 = cbase + (p * GL + gl) * VEC;
    if constexpr (CLAMP) {
      const bool ok = c0 < C;  // C % VEC == 0 (host)
      float t[VEC];
      load_vec<VEC>(xrow + (ok ? c0 : 0), t);
#pragma unroll
      for (int i = 0; i < VEC; ++i) xv[p][i] = ok ? t[i] : 0.f;
    } else {
      load_vec<VEC>(xrow + c0, xv[p]);
    }
  }
}

template <int VEC, int NP, int GL, int MAXH>
__device__ __forceinline__ void ns_load_u(const double* __restrict__ Ub, int cbase, int gl,
                                          double (&u)[NP][VEC][MAXH]) {
  const double* __restrict__ base = Ub + (int64_t)(cbase + gl * VEC) * MAXH;
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int i = 0; i < VEC; ++i)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) u[p][i][h] = base[(p * GL * VEC + i) * MAXH + h];
}

template <int VEC, int NP, int MAXH>
__device__ __forceinline__ void ns_dot(const float (&xv)[NP][VEC], const double (&u)[NP][VEC][MAXH],
                                       double (&acc)[MAXH]) {
#pragma unroll
  for (int p = 0; p < NP; ++p)
#pragma unroll
    for (int i = 0; i < VEC; ++i)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) acc[h] = fma((double)xv[p][i], u[p][i][h], acc[h]);
}

// reduce over the GL lanes of a row and store cs[row, :H] from lane gl == 0
// (branch-free buffer stores; other lanes and heads past H pass kBufNone)
template <int GL, int MAXH>
__device__ __forceinline__ void ns_store(double (&acc)[MAXH], const double (&vb)[MAXH], int gl, int H, bool live,
                                         __amdgpu_buffer_rsrc_t rcs, int64_t row) {
#pragma unroll
  for (int o = 1; o < GL; o <<= 1)
#pragma unroll
    for (int h = 0; h < MAXH; ++h) acc[h] += __shfl_xor(acc[h], o);
  const bool st = gl == 0 && live;
#pragma unroll
  for (int h = 0; h < MAXH; ++h)
    buf_store_f64(rcs, (st && h < H) ? (uint32_t)((row * H + h) * 8) : kBufNone, acc[h] + vb[h]);
}

// One chunk per row: U[b] sits in registers and each wave keeps kNsDepth row
// groups in flight (a ring of kNsDepth register buffers, the loop unrolled by
// it so every index is static): a group is reduced, then its buffer refilled
// with the group kNsDepth steps ahead.  Depth 2 / 4 / 6 (with 4 / 8 / 12 key-sum
// rows in flight): reference attention RHS 0.1423 / 0.1429 / 0.1437 ms — the
// ~20 us of the launch is not the prefetch depth.
// Prefetch addresses past the block's rows clamp to its last row (a cache-line
// hit, no extra HBM traffic).  ns_first_rows issues the first kNsDepth groups,
// before U exists when the block forms U itself (node_scores_fused_kernel).
#ifndef GNPDE_NS_DEPTH
#define GNPDE_NS_DEPTH 2  // deeper rings measured no faster (above)
#endif
// depth per head count: GNPDE_NS_DEPTH groups of NPV floats, capped at 64 floats of ring
template <int MAXH>
constexpr int ns_depth() {
  constexpr int d = 64 / node_scores_npv<MAXH>();
  return d < 2 ? 2 : (d > GNPDE_NS_DEPTH ? GNPDE_NS_DEPTH : d);
}

template <int VEC, int GL, int MAXH>
using NsRing = float[ns_depth<MAXH>()][node_scores_npv<MAXH>() / VEC][VEC];

template <int VEC, int GL, int MAXH, bool CLAMP>
__device__ __forceinline__ void ns_first_rows(const float* __restrict__ xb, int64_t n0, int64_t n1, int C,
                                              int64_t ldx, int g, int gl, int wv, NsRing<VEC, GL, MAXH>& xr) {
  constexpr int G = kWave / GL;
  constexpr int NP = node_scores_npv<MAXH>() / VEC;
  const int64_t step = (int64_t)kWavesPerBlock * G;
  const int64_t last = n1 - 1, nb = n0 + wv * G;
  constexpr int kNsDepth = ns_depth<MAXH>();
#pragma unroll
  for (int d = 0; d < kNsDepth; ++d)
    ns_load_x<VEC, NP, GL, CLAMP>(xb + min(nb + g + d * step, last) * ldx, 0, gl, C, xr[d]);
}

template <int VEC, int GL, int MAXH, bool CLAMP, bool PRELOADED = false>
__device__ __forceinline__ void ns_block_resident(const double* __restrict__ Ub, const float* __restrict__ xb,
                                                  __amdgpu_buffer_rsrc_t rcs, int64_t n0, int64_t n1, int C,
                                                  int64_t ldx, int H, int Cp, int g, int gl, int wv,
                                                  NsRing<VEC, GL, MAXH>& xr) {
  constexpr int G = kWave / GL;
  constexpr int NP = node_scores_npv<MAXH>() / VEC;
  const int64_t step = (int64_t)kWavesPerBlock * G;
  const int64_t last = n1 - 1;
  constexpr int kNsDepth = ns_depth<MAXH>();
  if constexpr (!PRELOADED) ns_first_rows<VEC, GL, MAXH, CLAMP>(xb, n0, n1, C, ldx, g, gl, wv, xr);
  double u[NP][VEC][MAXH];
  ns_load_u<VEC, NP, GL, MAXH>(Ub, 0, gl, u);
  double vb[MAXH];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) vb[h] = Ub[Cp * MAXH + h];
  for (int64_t nb = n0 + wv * G; nb < n1; nb += kNsDepth * step) {
#pragma unroll
    for (int d = 0; d < kNsDepth; ++d) {
      const int64_t nr = nb + d * step + g;
      double acc[MAXH];
#pragma unroll
      for (int h = 0; h < MAXH; ++h) acc[h] = 0.0;
      ns_dot<VEC, NP, MAXH>(xr[d], u, acc);
      ns_store<GL, MAXH>(acc, vb, gl, H, nr < n1, rcs, nr);
      ns_load_x<VEC, NP, GL, CLAMP>(xb + min(nr + kNsDepth * step, last) * ldx, 0, gl, C, xr[d]);
    }
  }
}

// uv: per batch element U[Cp][MAXH] | v[MAXH] (key_projection_kernel)
template <int VEC, int GL, int MAXH>
__global__ __launch_bounds__(256) void node_scores_kernel(const float* __restrict__ x, int64_t B, int64_t N, int C,
                                                           int64_t ldx, int H, int nch, const double* __restrict__ uv,
                                                           double* __restrict__ cs, int64_t rows_per_block) {
  constexpr int G = kWave / GL;
  constexpr int NPV = node_scores_npv<MAXH>();
  constexpr int NP = NPV / VEC;
  constexpr int CW = GL * NPV;
  static_assert(NP >= 1, "node_scores: VEC wider than the per-lane column budget");
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int g = lane / GL, gl = lane % GL;
  const int64_t n0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t n1 = min(N, n0 + rows_per_block);
  const int64_t step = (int64_t)kWavesPerBlock * G;
  const bool ragged = C != nch * CW;
  const int Cp = nch * CW;
  for (int64_t b = blockIdx.y; b < B; b += gridDim.y) {
    const float* __restrict__ xb = x + b * N * ldx;
    const double* __restrict__ Ub = uv + b * ((int64_t)Cp * MAXH + MAXH);
    const __amdgpu_buffer_rsrc_t rcs = buf_rsrc(cs + b * N * H);
    if (nch == 1) {
      NsRing<VEC, GL, MAXH> xr;
      if (ragged)
        ns_block_resident<VEC, GL, MAXH, true>(Ub, xb, rcs, n0, n1, C, ldx, H, Cp, g, gl, wv, xr);
      else
        ns_block_resident<VEC, GL, MAXH, false>(Ub, xb, rcs, n0, n1, C, ldx, H, Cp, g, gl, wv, xr);
    } else {
      double vb[MAXH];
#pragma unroll
      for (int h = 0; h < MAXH; ++h) vb[h] = Ub[Cp * MAXH + h];
      for (int64_t nb = n0 + wv * G; nb < n1; nb += step) {
        const int64_t nr = nb + g;
        const float* xrow = xb + min(nr, N - 1) * ldx;
        double acc[MAXH];
#pragma unroll
        for (int h = 0; h < MAXH; ++h) acc[h] = 0.0;
        for (int ch = 0; ch < nch; ++ch) {
          double u[NP][VEC][MAXH];
          float xc[NP][VEC];
          ns_load_x<VEC, NP, GL, true>(xrow, ch * CW, gl, C, xc);
          ns_load_u<VEC, NP, GL, MAXH>(Ub, ch * CW, gl, u);
          ns_dot<VEC, NP, MAXH>(xc, u, acc);
        }
        ns_store<GL, MAXH>(acc, vb, gl, H, nr < n1, rcs, nr);
      }
    }
  }
}

// Node scores with the key projection formed by every workgroup itself (no
// separate key_projection launch: it was one latency-bound workgroup, 6.4 us on
// G-arxiv, between two bandwidth-bound launches).  Each block issues its first
// two row groups of x, then sums the keysum tile shares of S (thread (tg, d):
// tiles tg, tg + TG, ... in order, then the TG group sums in order — the same
// fixed order in every block, so every block forms the same U bit for bit),
// forms U = Wq^T S / sqrt(dk) and v = bq . S / sqrt(dk) into LDS and streams its
// rows with U[b] in registers.  One chunk per row (nch == 1), one batch element
// per grid row (gridDim.y == B).
constexpr int kNsfPre = 16;    // Wq values per U output held in registers (dk <= 16)
constexpr int kNsfLoads = 32;  // tile shares in flight per thread
#ifndef GNPDE_NSF_OUTS
#define GNPDE_NSF_OUTS 1  // 4 (the 8-head Cora shape's U in one load round): 18.9 against 16.2 us
#endif
constexpr int kNsfOuts = GNPDE_NSF_OUTS;
constexpr int64_t kNsSplitRows = 50000;  // below: key_projection_kernel + node_scores_kernel  // U outputs per thread with their Wq values in registers

template <int VEC, int GL, int MAXH, bool CLAMP>
__global__ __launch_bounds__(256) void node_scores_fused_kernel(const float* __restrict__ x, int64_t N, int C,
                                                                 int64_t ldx, int H, const double* __restrict__ part,
                                                                 int ntiles, const float* __restrict__ Wq,
                                                                 const float* __restrict__ bq, int att,
                                                                 double* __restrict__ cs, int64_t rows_per_block) {
  constexpr int NPV = node_scores_npv<MAXH>();
  constexpr int Cp = GL * NPV;
  extern __shared__ __attribute__((aligned(16))) double nsf_lds[];  // S[att] | red[256] | U[Cp*MAXH] | v[MAXH]
  double* S = nsf_lds;
  double* red = S + att;
  double* U = red + kBlock;
  const int tid = threadIdx.x;
  const int lane = tid & 63, wv = tid >> 6;
  const int g = lane / GL, gl = lane % GL;
  const int64_t b = blockIdx.y;
  const int64_t n0 = (int64_t)blockIdx.x * rows_per_block;
  const int64_t n1 = min(N, n0 + rows_per_block);
  const float* __restrict__ xb = x + b * N * ldx;
  NsRing<VEC, GL, MAXH> xr;
  ns_first_rows<VEC, GL, MAXH, CLAMP>(xb, n0, n1, C, ldx, g, gl, wv, xr);
  // this thread's operands of U, loaded before S is known: KO outputs (c, h) =
  // (t / MAXH, t % MAXH) at t = o * kBlock + tid, and the v outputs (c = Cp) in the
  // first MAXH threads' extra slot (KO <= kNsfOuts; more outputs take the loop below)
  constexpr int KO = (Cp * MAXH + kBlock - 1) / kBlock;
  const int dk = att / H;
  const bool pre = dk <= kNsfPre && KO <= kNsfOuts && Cp * MAXH == KO * kBlock;
  float wq[KO <= kNsfOuts ? KO + 1 : 1][kNsfPre];
  if constexpr (KO <= kNsfOuts) {
#pragma unroll
    for (int o = 0; o <= KO; ++o) {
      const int t = o < KO ? o * kBlock + tid : Cp * MAXH + tid;
      const int c = t / MAXH, h = t - c * MAXH;
      const bool ok = pre && (o < KO || tid < MAXH) && h < H && (c < C || c == Cp);
#pragma unroll
      for (int d = 0; d < kNsfPre; ++d) {
        const int dd = h * dk + min(d, dk - 1);
        wq[o][d] = (ok && d < dk) ? (c == Cp ? bq[dd] : Wq[(int64_t)dd * C + c]) : 0.f;
      }
    }
  }
  // S = sum over the tile shares: every share of the thread in flight at once
  const double* __restrict__ pb = part + b * (int64_t)ntiles * att;
  const int DW = min(att, kBlock), TG = kBlock / DW;
  const int tg = tid / DW, dl = tid - tg * DW;
  for (int d0 = 0; d0 < att; d0 += DW) {
    const int d = d0 + dl;
    double acc = 0.0;
    if (tg < TG && d < att) {
      for (int t0 = tg; t0 < ntiles; t0 += kNsfLoads * TG) {
        double v[kNsfLoads];
#pragma unroll
        for (int k = 0; k < kNsfLoads; ++k) v[k] = pb[(int64_t)min(t0 + k * TG, ntiles - 1) * att + d];
#pragma unroll
        for (int k = 0; k < kNsfLoads; ++k)
          if (t0 + k * TG < ntiles) acc += v[k];
      }
    }
    red[tid] = acc;
    __syncthreads();
    if (tid < DW && d0 + tid < att) {
      double sum = 0.0;
      for (int q = 0; q < TG; ++q) sum += red[q * DW + tid];
      S[d0 + tid] = sum;
    }
    __syncthreads();
  }
  // U[c][h] (c < Cp; zero past C and H) and v[h] (row c = Cp)
  const double inv = 1.0 / sqrt((double)dk);
  if (KO <= kNsfOuts && pre) {
#pragma unroll
    for (int o = 0; o < (KO <= kNsfOuts ? KO + 1 : 1); ++o) {
      const int t = o < KO ? o * kBlock + tid : Cp * MAXH + tid;
      if (t < (Cp + 1) * MAXH && (o < KO || tid < MAXH)) {
        const int c = t / MAXH, h = t - c * MAXH;
        double a = 0.0;
#pragma unroll
        for (int d = 0; d < kNsfPre; ++d)
          if (d < dk && h < H) a = fma((double)wq[o][d], S[h * dk + d], a);
        U[t] = a * inv;
      }
    }
  } else {
    for (int t = tid; t < (Cp + 1) * MAXH; t += kBlock) {
      const int c = t / MAXH, h = t - c * MAXH;
      double a = 0.0;
      if (h < H && (c < C || c == Cp)) {
        const int d0 = h * dk;
#pragma unroll 8
        for (int d = 0; d < dk; ++d)
          a = fma((double)(c == Cp ? bq[d0 + d] : Wq[(int64_t)(d0 + d) * C + c]), S[d0 + d], a);
      }
      U[t] = a * inv;
    }
  }
  __syncthreads();
  const __amdgpu_buffer_rsrc_t rcs = buf_rsrc(cs + b * N * H);
  ns_block_resident<VEC, GL, MAXH, CLAMP, true>(U, xb, rcs, n0, n1, C, ldx, H, Cp, g, gl, wv, xr);
}

// S[b][d] = the sum of the tile shares part[b][tile][d]: the key sum of
// gnpde_ref_keysum_f32, handed to the caller (a sharded solve all-reduces it over the
// column stripes before the node scores).  One wavefront per (b, d): lane l sums tiles
// l, l + 64, ... in order, then a fixed xor tree (one thread walking all ~256 tiles in
// a chain of dependent loads took 62 us on G-arxiv, the sharded reference RHS's
// slowest launch).
__global__ __launch_bounds__(256) void keysum_reduce_kernel(const double* __restrict__ part, int ntiles, int att,
                                                             int64_t B, double* __restrict__ S) {
  const int64_t i = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (i >= B * att) return;
  const int lane = threadIdx.x & 63;
  const int64_t b = i / att, d = i - b * att;
  const double* __restrict__ pb = part + b * (int64_t)ntiles * att + d;
  double acc = 0.0;
  for (int t = lane; t < ntiles; t += kWave) acc += pb[(int64_t)t * att];
#pragma unroll
  for (int o = kWave / 2; o > 0; o >>= 1) acc += __shfl_xor(acc, o);
  if (lane == 0) S[i] = acc;
}

// ------------------------------------------------------------------ host helpers
static int pow2_at_least(int v, int cap) {
  int p = 1;
  while (p < v && p < cap) p <<= 1;
  return p;
}

static int keysum_vec(int64_t C, const float* x, int64_t ldx) {
  if (C % 4 == 0 && ldx % 4 == 0 && aligned16(x)) return 4;
  if (C % 2 == 0 && ldx % 2 == 0 && aligned8(x)) return 2;
  return 1;
}

// tiles of rows for the partial column sums (independent of the vector width):
// about kKeysumTilesTarget over the launch, at least one row per row slot
static int keysum_tiles_target() {
  if constexpr (!GNPDE_EXPERIMENTS) return kKeysumTilesTarget;
  static const int t = [] {
    const char* e = std::getenv("GNPDE_KEYSUM_TILES");  // tuning knob (experiment builds)
    const int v = e ? std::atoi(e) : 0;
    return v >= 8 && v <= 4096 ? v : kKeysumTilesTarget;
  }();
  return t;
}

static void keysum_tiles(int64_t B, int64_t N, int rpb, int* rows_per_tile, int* ntiles) {
  const int64_t per_batch = std::max<int64_t>(1, keysum_tiles_target() / B);
  const int64_t rpt = std::max<int64_t>(ceil_div(N, per_batch), rpb);
  *rows_per_tile = (int)rpt;
  *ntiles = (int)ceil_div(N, rpt);
}

// keysum geometry: 16-byte (or narrower) loads, TPR threads per row
static void keysum_geometry(int64_t C, const float* x, int64_t ldx, int* vec, int* tpr) {
  *vec = keysum_vec(C, x, ldx);
  *tpr = pow2_at_least((int)ceil_div(C, *vec), kKeysumBlock);
}

template <int MAXH>
static void launch_stats(unsigned grid, int GL, hipStream_t s, const int4* it, int n, const int* gidx, int gid,
                         const ScoreArgs& sa, double* m, float* rl, float* mr, double* partials) {
  if (GL == 8)
    stats_kernel<MAXH, 8><<<grid, kBlock, 0, s>>>(it, n, gidx, gid, sa, m, rl, mr, partials);
  else
    stats_kernel<MAXH, 64><<<grid, kBlock, 0, s>>>(it, n, gidx, gid, sa, m, rl, mr, partials);
}

// node_scores geometry: VEC, MAXH (= Hp), lanes per row GL (8..64) so one
// chunk of CW = GL*NPV columns covers the row when it can, nch chunks.
struct NsGeom {
  int vec, maxh, GL, CW, nch;
};

static NsGeom ns_geometry(int vec, int64_t C, int64_t H) {
  NsGeom g;
  g.maxh = H <= 1 ? 1 : H <= 2 ? 2 : H <= 4 ? 4 : H <= 8 ? 8 : 16;
  const int npv = kNodeScoreURegs / g.maxh;
  g.vec = (vec == 4 && npv >= 4) ? 4 : 1;
  g.GL = std::max(8, pow2_at_least((int)ceil_div(C, npv), 64));
  g.CW = g.GL * npv;
  g.nch = (int)ceil_div(C, g.CW);
  return g;
}

// doubles of U[Cp][MAXH] | v[MAXH] per batch element
static int64_t ns_uv_doubles(const NsGeom& ge) { return (int64_t)ge.nch * ge.CW * ge.maxh + ge.maxh; }

template <int VEC, int MAXH>
static void launch_node_scores(dim3 grid, const NsGeom& ge, hipStream_t s, const float* x, int64_t B, int64_t N, int C,
                               int64_t ldx, int H, const double* uv, double* cs, int64_t rpb) {
  const int n = ge.nch;
  if (ge.GL <= 8)
    node_scores_kernel<VEC, 8, MAXH><<<grid, kBlock, 0, s>>>(x, B, N, C, ldx, H, n, uv, cs, rpb);
  else if (ge.GL <= 16)
    node_scores_kernel<VEC, 16, MAXH><<<grid, kBlock, 0, s>>>(x, B, N, C, ldx, H, n, uv, cs, rpb);
  else if (ge.GL <= 32)
    node_scores_kernel<VEC, 32, MAXH><<<grid, kBlock, 0, s>>>(x, B, N, C, ldx, H, n, uv, cs, rpb);
  else
    node_scores_kernel<VEC, 64, MAXH><<<grid, kBlock, 0, s>>>(x, B, N, C, ldx, H, n, uv, cs, rpb);
}

// rows per block sized for ~1024 wavefronts over the whole launch (one block per
// CU, one wave per SIMD streaming its rows with two row groups in flight): the
// kernel holds U[b] in registers, and the whole grid runs in one round (G-arxiv,
// 87 MB: 15.4-15.5 us against 16.0-16.1 with 2048 wavefronts, three A/B pairs;
// 4096 waves left a 1.7-round tail: 26.9 us)
static void launch_node_scores_any(hipStream_t s, const NsGeom& ge, const float* x, int64_t B, int64_t N, int C,
                                   int64_t ldx, int H, const double* uv, double* cs) {
  const int G = kWave / ge.GL;
  const int64_t groups = ceil_div(N, (int64_t)G);
  const int64_t waves_per_batch = std::max<int64_t>(1, 1024 / B);
  const int64_t iters = std::max<int64_t>(1, ceil_div(groups, waves_per_batch));
  const int64_t rpb = (int64_t)kWavesPerBlock * G * iters;
  const dim3 grid((unsigned)ceil_div(N, rpb), (unsigned)std::min<int64_t>(B, 65535));
#define GNPDE_NS(V, M) launch_node_scores<V, M>(grid, ge, s, x, B, N, C, ldx, H, uv, cs, rpb)
  if (ge.vec == 4) {
    switch (ge.maxh) {
      case 1: GNPDE_NS(4, 1); break;
      case 2: GNPDE_NS(4, 2); break;
      case 4: GNPDE_NS(4, 4); break;
      default: GNPDE_NS(4, 8); break;
    }
  } else {
    switch (ge.maxh) {
      case 1: GNPDE_NS(1, 1); break;
      case 2: GNPDE_NS(1, 2); break;
      case 4: GNPDE_NS(1, 4); break;
      case 8: GNPDE_NS(1, 8); break;
      default: GNPDE_NS(1, 16); break;
    }
  }
#undef GNPDE_NS
}

// Experiment builds: GNPDE_NS_FUSED=0 keeps the separate key_projection launch.
static bool ns_fused_enabled() {
  if constexpr (!GNPDE_EXPERIMENTS) return true;
  static const bool v = [] {
    const char* e = std::getenv("GNPDE_NS_FUSED");
    return !(e && e[0] == '0');
  }();
  return v;
}

template <int VEC, int GL, int MAXH>
static void launch_nsf(dim3 grid, size_t lds, bool ragged, hipStream_t s, const float* x, int64_t N, int C,
                       int64_t ldx, int H, const double* part, int ntiles, const float* Wq, const float* bq, int att,
                       double* cs, int64_t rpb) {
  if (ragged)
    node_scores_fused_kernel<VEC, GL, MAXH, true><<<grid, kBlock, lds, s>>>(x, N, C, ldx, H, part, ntiles, Wq, bq, att,
                                                                          cs, rpb);
  else
    node_scores_fused_kernel<VEC, GL, MAXH, false><<<grid, kBlock, lds, s>>>(x, N, C, ldx, H, part, ntiles, Wq, bq,
                                                                           att, cs, rpb);
}

// the same grid as launch_node_scores_any (~1024 wavefronts), one grid row per batch element
static void launch_node_scores_fused(hipStream_t s, const NsGeom& ge, const float* x, int64_t B, int64_t N, int C,
                                     int64_t ldx, int H, const double* part, int ntiles, const float* Wq,
                                     const float* bq, int att, double* cs) {
  const int G = kWave / ge.GL;
  const int64_t groups = ceil_div(N, (int64_t)G);
  const int64_t waves_per_batch = std::max<int64_t>(1, 1024 / B);
  const int64_t iters = std::max<int64_t>(1, ceil_div(groups, waves_per_batch));
  const int64_t rpb = (int64_t)kWavesPerBlock * G * iters;
  const dim3 grid((unsigned)ceil_div(N, rpb), (unsigned)B);
  const size_t lds = sizeof(double) * (size_t)(att + kBlock + (ge.CW + 1) * ge.maxh);
  const bool ragged = C != ge.CW;
#define GNPDE_NSF(V, GLV, M) \
  launch_nsf<V, GLV, M>(grid, lds, ragged, s, x, N, C, ldx, H, part, ntiles, Wq, bq, att, cs, rpb)
#define GNPDE_NSF_GL(V, M)                    \
  do {                                        \
    if (ge.GL <= 8) GNPDE_NSF(V, 8, M);       \
    else if (ge.GL <= 16) GNPDE_NSF(V, 16, M); \
    else if (ge.GL <= 32) GNPDE_NSF(V, 32, M); \
    else GNPDE_NSF(V, 64, M);                 \
  } while (0)
  if (ge.vec == 4) {
    switch (ge.maxh) {
      case 1: GNPDE_NSF_GL(4, 1); break;
      case 2: GNPDE_NSF_GL(4, 2); break;
      case 4: GNPDE_NSF_GL(4, 4); break;
      default: GNPDE_NSF_GL(4, 8); break;
    }
  } else {
    switch (ge.maxh) {
      case 1: GNPDE_NSF_GL(1, 1); break;
      case 2: GNPDE_NSF_GL(1, 2); break;
      case 4: GNPDE_NSF_GL(1, 4); break;
      case 8: GNPDE_NSF_GL(1, 8); break;
      default: GNPDE_NSF_GL(1, 16); break;
    }
  }
#undef GNPDE_NSF_GL
#undef GNPDE_NSF
}

static unsigned edge_grid(int64_t nnz) {
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nnz, kBlock), 16384));
}

// a block takes kWavesPerBlock * 64 consecutive edges per pass (T per team)
static unsigned team_grid(int64_t nnz, const Team& tm) {
  const int64_t per_block = (int64_t)kWavesPerBlock * (kWave / tm.T) * tm.T;
  return (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(nnz, per_block), 32768));
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_softmax_stats_f32(const int32_t* items, int64_t n_items, const int32_t* heavy, int64_t n_heavy,
                            const int32_t* gidx, int group_is_dst, int mode, int64_t heads, int64_t dk,
                            const double* cs, const float* q, const float* k, int64_t ldqk, float score_p0,
                            float score_p1, double* m, float* rl, float* mr, double* partials,
                            void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE((m && rl) || mr, GNPDE_EINVAL, "softmax_stats: no output (m/rl or the packed records)");
  GNPDE_REQUIRE(n_heavy == 0 || partials, GNPDE_EINVAL, "softmax_stats: hub groups need partials");
  if (n_items == 0) return GNPDE_OK;
  GNPDE_REQUIRE(items && gidx, GNPDE_EINVAL, "softmax_stats: NULL items/gidx");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  hipStream_t s = as_stream(stream);
  const int4* it = reinterpret_cast<const int4*>(items);
  const Team tm = team_geometry(sa);
  if (tm.T > 0) {
    const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * (kWave / tm.T));
    stats_team_kernel<4><<<grid, kBlock, 0, s>>>(it, (int)n_items, gidx, group_is_dst, sa, tm, m, rl, mr, partials);
    GNPDE_LAUNCH_CHECK();
  } else {
  const int GL = 8;  // lanes per item
  const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * (kWave / GL));
  if (heads <= 1)
    launch_stats<1>(grid, GL, s, it, (int)n_items, gidx, group_is_dst, sa, m, rl, mr, partials);
  else if (heads <= 2)
    launch_stats<2>(grid, GL, s, it, (int)n_items, gidx, group_is_dst, sa, m, rl, mr, partials);
  else if (heads <= 4)
    launch_stats<4>(grid, GL, s, it, (int)n_items, gidx, group_is_dst, sa, m, rl, mr, partials);
  else if (heads <= 8)
    launch_stats<8>(grid, GL, s, it, (int)n_items, gidx, group_is_dst, sa, m, rl, mr, partials);
  else
    launch_stats<16>(grid, GL, s, it, (int)n_items, gidx, group_is_dst, sa, m, rl, mr, partials);
  GNPDE_LAUNCH_CHECK();
  }
  return launch_stats_fixup(reinterpret_cast<const int4*>(heavy), n_heavy, (int)heads, partials, m, rl, mr, s);
}

int gnpde_attn_weights_f32(const int32_t* rowidx, const int32_t* col, int64_t nnz, int norm_idx, int mode,
                           int64_t heads, int64_t dk, const double* cs, const float* q, const float* k, int64_t ldqk,
                           float score_p0, float score_p1, const double* m, const float* rl, float* w_out,
                           void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE(norm_idx == 0 || norm_idx == 1, GNPDE_EINVAL, "attn_weights: norm_idx must be 0 or 1");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowidx && col && m && rl && w_out, GNPDE_EINVAL, "attn_weights: NULL pointer");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  Team tm = team_geometry(sa);
  if ((uint64_t)nnz * 4 >= kBufRecords) tm.T = 0;  // buffer-store offsets are 32-bit
  if (tm.T > 0)
    attn_team_kernel<4, false><<<team_grid(nnz, tm), kBlock, 0, as_stream(stream)>>>(rowidx, col, nullptr, nnz, norm_idx,
                                                                                    sa, tm, m, rl, w_out);
  else
    attn_weights_kernel<<<edge_grid(nnz), kBlock, 0, as_stream(stream)>>>(rowidx, col, nnz, norm_idx, sa, m, rl,
                                                                          w_out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_edge_attention_f32(const int32_t* rowidx, const int32_t* col, const int32_t* perm, int64_t nnz,
                             int norm_idx, int mode, int64_t heads, int64_t dk, const double* cs, const float* q,
                             const float* k, int64_t ldqk, float score_p0, float score_p1, const double* m,
                             const float* rl, float* att, void* stream) {
  int rc = check_score_args(mode, heads, dk, cs, q, k);
  if (rc) return rc;
  GNPDE_REQUIRE(norm_idx == 0 || norm_idx == 1, GNPDE_EINVAL, "edge_attention: norm_idx must be 0 or 1");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowidx && col && perm && m && rl && att, GNPDE_EINVAL, "edge_attention: NULL pointer");
  const ScoreArgs sa = make_score_args(mode, heads, dk, cs, q, k, ldqk, score_p0, score_p1);
  Team tm = team_geometry(sa);
  if ((uint64_t)nnz * heads * 4 >= kBufRecords) tm.T = 0;  // buffer-store offsets are 32-bit
  if (tm.T > 0)
    attn_team_kernel<4, true><<<team_grid(nnz, tm), kBlock, 0, as_stream(stream)>>>(rowidx, col, perm, nnz, norm_idx, sa,
                                                                                   tm, m, rl, att);
  else
    edge_attention_kernel<<<edge_grid(nnz), kBlock, 0, as_stream(stream)>>>(rowidx, col, perm, nnz, norm_idx, sa, m,
                                                                            rl, att);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

size_t gnpde_keysum_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t att) {
  // most tiles: 4-byte loads (fewest rows per slot), whatever x's alignment
  int rpt, ntiles;
  keysum_tiles(B, N, kKeysumBlock / pow2_at_least((int)C, kKeysumBlock), &rpt, &ntiles);
  // tile shares of S [B][ntiles][att] | U, v per batch element: Cp*Hp = nch*GL*32 < 16*C + 2048, Hp <= 16
  return sizeof(double) * (size_t)(B * ntiles * att + B * (16 * C + 2048 + 16));
}

// The key-sum launch of the reference scores: part[b][tile][att] tile shares of
// S = Wk xbar + E bk (keysum_partial_kernel).  Returns the tile count.
static int ref_keysum_launch(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                             const float* Wk, const float* bk, int64_t att, double* part, hipStream_t s, int* ntiles_out) {
  int vec, tpr, rpt, ntiles;
  keysum_geometry(C, x, ldx, &vec, &tpr);
  const int rpb = kKeysumBlock / tpr;
  keysum_tiles(B, N, rpb, &rpt, &ntiles);
  const size_t shm = sizeof(double) * (size_t)(rpb + 1) * (C + 1);
  GNPDE_REQUIRE(shm <= 64 * 1024, GNPDE_EUNSUPPORTED, "ref_scores: C too large");
  const dim3 g1((unsigned)ntiles, (unsigned)B);
#define GNPDE_KS(V) keysum_partial_kernel<V><<<g1, kKeysumBlock, shm, s>>>(x, N, (int)C, ldx, indeg, Wk, bk, (int)att, rpt, tpr, \
                                                         ntiles, part)
  if (vec == 4)
    GNPDE_KS(4);
  else if (vec == 2)
    GNPDE_KS(2);
  else
    GNPDE_KS(1);
#undef GNPDE_KS
  GNPDE_LAUNCH_CHECK();
  *ntiles_out = ntiles;
  return GNPDE_OK;
}

// The node-score launches from the tile shares `part` (ntiles of them per batch
// element; ntiles = 1: S itself): U = Wq^T S / sqrt(dk), v, cs = x U + v.
static int ref_node_scores_launch(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const float* Wq,
                                  const float* bq, int64_t att, int64_t heads, const double* part, int ntiles,
                                  double* cs, double* uv, hipStream_t s) {
  int vec, tpr;
  keysum_geometry(C, x, ldx, &vec, &tpr);
  const NsGeom ge = ns_geometry(vec, C, heads);
  const int64_t cp = (int64_t)ge.nch * ge.CW;
  GNPDE_REQUIRE(ns_uv_doubles(ge) <= 16 * C + 2048 + 16, GNPDE_EUNSUPPORTED, "ref_scores: node-score geometry");
  // small graphs (B N < kNsSplitRows: the launch is a handful of rows per workgroup) take
  // the projection once, in its own workgroup, instead of in every node-score workgroup:
  // Cora-sized 8-head scores 6.3 + 6.7 us against 16.2 us fused
  if (ge.nch == 1 && att <= 1024 && B <= 65535 && B * N >= kNsSplitRows && ns_fused_enabled()) {
    // every node-score workgroup forms U itself (node_scores_fused_kernel): two launches
    launch_node_scores_fused(s, ge, x, B, N, (int)C, ldx, (int)heads, part, ntiles, Wq, bq, (int)att, cs);
    GNPDE_LAUNCH_CHECK();
    return GNPDE_OK;
  }
  const size_t shm2 = sizeof(double) * (size_t)(att + kKeysumBlock);
  key_projection_kernel<<<(unsigned)B, kKeysumBlock, shm2, s>>>(part, ntiles, (int)C, Wq, bq, (int)att, (int)heads,
                                                                 (int)cp, ge.maxh, uv);
  GNPDE_LAUNCH_CHECK();
  launch_node_scores_any(s, ge, x, B, N, (int)C, ldx, (int)heads, uv, cs);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

static int ref_scores_check(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, int64_t att, int64_t heads,
                            size_t workspace_bytes) {
  GNPDE_REQUIRE(B >= 1 && N >= 1 && C >= 1 && ldx >= C, GNPDE_EINVAL, "ref_scores: bad sizes");
  GNPDE_REQUIRE(heads >= 1 && heads <= 16 && att % heads == 0, GNPDE_EUNSUPPORTED,
                "ref_scores: heads must divide attention_dim and be <= 16");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_keysum_workspace_bytes(B, N, C, att), GNPDE_EINVAL,
                "ref_scores: workspace too small");
  GNPDE_REQUIRE(att <= 4096, GNPDE_EUNSUPPORTED, "ref_scores: attention_dim too large");
  GNPDE_REQUIRE(B <= 65535, GNPDE_EUNSUPPORTED, "ref_scores: batch too large");
  GNPDE_REQUIRE((uint64_t)N * heads * 8 < kBufRecords, GNPDE_EUNSUPPORTED, "ref_scores: N*heads too large");
  return GNPDE_OK;
}

int gnpde_ref_scores_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                         const float* Wq, const float* bq, const float* Wk, const float* bk, int64_t att,
                         int64_t heads, double* cs, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(x && indeg && Wq && bq && Wk && bk && cs && workspace, GNPDE_EINVAL, "ref_scores: NULL pointer");
  int rc = ref_scores_check(x, B, N, C, ldx, att, heads, workspace_bytes);
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  int ntiles = 0;
  rc = ref_keysum_launch(x, B, N, C, ldx, indeg, Wk, bk, att, part, s, &ntiles);
  if (rc) return rc;
  return ref_node_scores_launch(x, B, N, C, ldx, Wq, bq, att, heads, part, ntiles, cs, part + B * ntiles * att, s);
}

int gnpde_ref_keysum_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                         const float* Wk, const float* bk, int64_t att, double* S, void* workspace,
                         size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(x && indeg && Wk && bk && S && workspace, GNPDE_EINVAL, "ref_keysum: NULL pointer");
  int rc = ref_scores_check(x, B, N, C, ldx, att, 1, workspace_bytes);
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  int ntiles = 0;
  rc = ref_keysum_launch(x, B, N, C, ldx, indeg, Wk, bk, att, part, s, &ntiles);
  if (rc) return rc;
  keysum_reduce_kernel<<<(unsigned)ceil_div(B * att, (int64_t)kWavesPerBlock), kBlock, 0, s>>>(part, ntiles, (int)att,
                                                                                                 B, S);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_ref_scores_from_keysum_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const double* S,
                                     const float* Wq, const float* bq, int64_t att, int64_t heads, double* cs,
                                     void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(x && S && Wq && bq && cs && workspace, GNPDE_EINVAL, "ref_scores_from_keysum: NULL pointer");
  int rc = ref_scores_check(x, B, N, C, ldx, att, heads, workspace_bytes);
  if (rc) return rc;
  return ref_node_scores_launch(x, B, N, C, ldx, Wq, bq, att, heads, S, 1, cs, static_cast<double*>(workspace),
                                as_stream(stream));
}

}  // extern "C"
