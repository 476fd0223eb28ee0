// backward.hip — gradients of the ODE right-hand side.
//
// The reference differentiates its RHS with torch autograd through a dense
// [B,N,N] matmul (src/function_laplacian_diffusion.py:39-58) and through the
// attention layer's gathers, [h,E,E] score matmul and torch_scatter softmax
// (src/function_transformer_attention.py:218-267, src/utils.py:116-127).  Here
// each piece of the chain rule is one pass over the graph:
//
//   * SDDMM     g_w[e] = a * <gf[src(e)], x[dst(e)]>      (d f / d w, f = a (A(w) x - x))
//               written straight into COO order (the layout of the weight
//               tensor the caller differentiates), divided over H heads when
//               the weights are a head mean;
//   * softmax   g_s[e,h] = att[e,h] * (g[e,h] - sum_{e' in grp} att[e',h] g[e',h])
//               per softmax group (fixed-order sum, fp64 accumulation);
//   * segment sums of per-edge values over the rows of a grouped CSR
//               (gradient of the node scores the edges gathered);
//   * weighted column sums  y[b,h,c] = sum_n w[b,n,h] x[b,n,c] (fp64 row
//               tiles + fixed-order tile reduction) for the key-sum scores;
//   * node-score input gradient  gx[n,c] += sum_h g_cs[n,h] U[c,h] + deg[n] g_xbar[c].
// No float atomics anywhere: every sum has a fixed order (bit-reproducible).
#include <algorithm>

#include "common.hpp"

namespace gnpde {

__device__ __forceinline__ float scale_of(const float* alpha, int alpha_sigmoid) {
  if (!alpha) return 1.f;
  const float a = *alpha;
  return alpha_sigmoid ? 1.0f / (1.0f + expf(-a)) : a;
}

// GL lanes per edge (team), G = 64/GL edges per wavefront pass; lane gl covers
// columns gl*VEC, gl*VEC + GL*VEC, ...; the team's partial dots meet in an xor tree.
template <int VEC, int GL>
__global__ __launch_bounds__(256) void sddmm_kernel(const int* __restrict__ rowidx, const int* __restrict__ col,
                                                     const int* __restrict__ perm, int64_t nnz, int C,
                                                     const float* __restrict__ gf, int64_t ldg,
                                                     const float* __restrict__ x, int64_t ldx,
                                                     const float* __restrict__ alpha, int alpha_sigmoid, int H,
                                                     float* __restrict__ g_out) {
  constexpr int G = kWave / GL;
  const int lane = threadIdx.x & 63;
  const int g = lane / GL, gl = lane % GL;
  const float a = scale_of(alpha, alpha_sigmoid) / (float)H;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t p0 = wave * G; p0 < nnz; p0 += nwaves * G) {
    const int64_t p = p0 + g;
    const bool live = p < nnz;
    const int64_t pc = live ? p : nnz - 1;
    const int r = rowidx[pc], c = col[pc];
    const float* __restrict__ gr = gf + (int64_t)r * ldg;
    const float* __restrict__ xr = x + (int64_t)c * ldx;
    float acc = 0.f;
    for (int cc = gl * VEC; cc < C; cc += GL * VEC) {
      float u[VEC], v[VEC];
      load_vec<VEC>(gr + cc, u);
      load_vec<VEC>(xr + cc, v);
#pragma unroll
      for (int t = 0; t < VEC; ++t) acc = fmaf(u[t], v[t], acc);
    }
#pragma unroll
    for (int o = 1; o < GL; o <<= 1) acc += __shfl_xor(acc, o);
    if (live && gl < H) g_out[(int64_t)perm[pc] * H + gl] = a * acc;
  }
}

// One wavefront per group (row of a grouped CSR), every head.
__global__ __launch_bounds__(256) void softmax_backward_kernel(const int* __restrict__ rowptr,
                                                                const int* __restrict__ perm, int64_t R, int H,
                                                                const float* __restrict__ att,
                                                                const float* __restrict__ g,
                                                                float* __restrict__ gs) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t r = wave; r < R; r += nwaves) {
    const int b = rowptr[r], e = rowptr[r + 1];
    for (int h = 0; h < H; ++h) {
      double d = 0.0;
      for (int p = b + lane; p < e; p += kWave) {
        const int64_t i = (int64_t)perm[p] * H + h;
        d = fma((double)att[i], (double)g[i], d);
      }
      d = wave_sum(d);
      for (int p = b + lane; p < e; p += kWave) {
        const int64_t i = (int64_t)perm[p] * H + h;
        gs[i] = (float)((double)att[i] * ((double)g[i] - d));
      }
    }
  }
}

// out[r, h] = sum over the row's edges of vals[perm[p]*H + h]  (fp64, fixed order)
__global__ __launch_bounds__(256) void segment_sum_kernel(const int* __restrict__ rowptr, const int* __restrict__ perm,
                                                           int64_t R, int H, const float* __restrict__ vals,
                                                           double* __restrict__ out) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t r = wave; r < R; r += nwaves) {
    const int b = rowptr[r], e = rowptr[r + 1];
    for (int h = 0; h < H; ++h) {
      double s = 0.0;
      for (int p = b + lane; p < e; p += kWave) s += (double)vals[(int64_t)perm[p] * H + h];
      s = wave_sum(s);
      if (lane == 0) out[r * H + h] = s;
    }
  }
}

// part[(b*H + h)][tile][c] = sum_{n in tile} w[b*N+n, h] * x[b*N+n, c]; [..][C] = sum w.
// One workgroup per (tile, b, h); TPR threads per row, RPB rows in flight.
__global__ __launch_bounds__(256) void wcolsum_partial_kernel(const float* __restrict__ x, int64_t N, int C,
                                                               int64_t ldx, const double* __restrict__ w, int H,
                                                               int rows_per_tile, int TPR, int ntiles,
                                                               double* __restrict__ part) {
  extern __shared__ __attribute__((aligned(16))) double red[];  // [RPB][C+1]
  const int tile = blockIdx.x, b = blockIdx.y, h = blockIdx.z;
  const int RPB = blockDim.x / TPR;
  const int rs = threadIdx.x / TPR, t = threadIdx.x % TPR;
  const int64_t n0 = (int64_t)tile * rows_per_tile;
  const int64_t n1 = min<int64_t>(N, n0 + rows_per_tile);
  const int64_t base = (int64_t)b * N;
  for (int c = t; c < C; c += TPR) {
    double acc = 0.0;
#pragma unroll 8
    for (int64_t n = n0 + rs; n < n1; n += RPB) acc = fma(w[(base + n) * H + h], (double)x[(base + n) * ldx + c], acc);
    red[rs * (C + 1) + c] = acc;
  }
  if (t == 0) {
    double ds = 0.0;
    for (int64_t n = n0 + rs; n < n1; n += RPB) ds += w[(base + n) * H + h];
    red[rs * (C + 1) + C] = ds;
  }
  __syncthreads();
  double* out = part + (((int64_t)b * H + h) * ntiles + tile) * (C + 1);
  for (int c = threadIdx.x; c <= C; c += blockDim.x) {
    double s = 0.0;
    for (int r = 0; r < RPB; ++r) s += red[r * (C + 1) + c];
    out[c] = s;
  }
}

// y[s][c] = sum_t part[s][t][c] (s = b*H + h), fixed order
__global__ __launch_bounds__(256) void wcolsum_tiles_kernel(const double* __restrict__ part, int ntiles, int C1,
                                                             double* __restrict__ y) {
  const int s = blockIdx.y;
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C1) return;
  double a = 0.0;
  for (int t = 0; t < ntiles; ++t) a += part[((int64_t)s * ntiles + t) * C1 + c];
  y[(int64_t)s * C1 + c] = a;
}

// gx[n,c] (+)= sum_h gcs[n,h] U[b][c][h] + deg[n] * gxbar[b][c]   (fp64 math)
__global__ __launch_bounds__(256) void score_input_grad_kernel(const double* __restrict__ gcs,
                                                                const double* __restrict__ U,
                                                                const int* __restrict__ deg,
                                                                const double* __restrict__ gxbar, int64_t N, int64_t R,
                                                                int C, int H, float* __restrict__ gx, int64_t ldgx,
                                                                int accumulate) {
  const int64_t total = R * C;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < total; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t n = i / C;
    const int c = (int)(i - n * C);
    const int64_t b = n / N;
    double s = (double)deg[n] * gxbar[b * C + c];
    for (int h = 0; h < H; ++h) s = fma(gcs[n * H + h], U[(b * C + c) * H + h], s);
    float* o = gx + n * ldgx + c;
    *o = accumulate ? (float)((double)*o + s) : (float)s;
  }
}

// out[p] = scale * w[perm[p]*H + h]   (one head of COO per-edge values in grouped-CSR order)
__global__ void gather_head_kernel(const float* __restrict__ w, int64_t nnz, int H, int h,
                                   const int* __restrict__ perm, float scale, float* __restrict__ out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x)
    out[p] = scale * w[(int64_t)perm[p] * H + h];
}

static int grid_n(int64_t n, int block = 256, int cap = 8192) {
  int64_t g = ceil_div(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

static int pow2_ge(int v, int cap) {
  int p = 1;
  while (p < v && p < cap) p <<= 1;
  return p;
}

constexpr int kWcolsumTiles = 256;

static void wcolsum_geometry(int64_t B, int64_t N, int* rpt, int* ntiles) {
  const int64_t per_b = std::max<int64_t>(1, kWcolsumTiles / B);
  const int64_t r = std::max<int64_t>(ceil_div(N, per_b), 1);
  *rpt = (int)r;
  *ntiles = (int)ceil_div(N, r);
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_sddmm_f32(const int32_t* rowidx, const int32_t* col, const int32_t* perm, int64_t nnz, int64_t C,
                    const float* gf, int64_t ldg, const float* x, int64_t ldx, const float* alpha, int alpha_sigmoid,
                    int heads, float* g_out, void* stream) {
  GNPDE_REQUIRE(C >= 1 && ldg >= C && ldx >= C && nnz >= 0, GNPDE_EINVAL, "sddmm: bad sizes");
  GNPDE_REQUIRE(heads >= 1 && heads <= kWave, GNPDE_EUNSUPPORTED, "sddmm: heads=%d not in [1,64]", heads);
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowidx && col && perm && gf && x && g_out, GNPDE_EINVAL, "sddmm: NULL pointer");
  const bool v4 = C % 4 == 0 && ldg % 4 == 0 && ldx % 4 == 0 && aligned16(gf) && aligned16(x);
  const int vec = v4 ? 4 : 1;
  // a team holds >= heads lanes: lane h < heads writes head h's copy of the gradient
  const int GL = std::max(std::max(8, pow2_ge(heads, 64)), pow2_ge((int)ceil_div(C, vec), 64));
  hipStream_t s = as_stream(stream);
  const int grid = grid_n(ceil_div(nnz, kWave / GL) * kWave, kBlock, 16384);
#define GNPDE_SD(V, L)                                                                                           \
  sddmm_kernel<V, L><<<grid, kBlock, 0, s>>>(rowidx, col, perm, nnz, (int)C, gf, ldg, x, ldx, alpha, alpha_sigmoid, \
                                             heads, g_out)
  if (vec == 4) {
    if (GL == 8) GNPDE_SD(4, 8);
    else if (GL == 16) GNPDE_SD(4, 16);
    else if (GL == 32) GNPDE_SD(4, 32);
    else GNPDE_SD(4, 64);
  } else {
    if (GL == 8) GNPDE_SD(1, 8);
    else if (GL == 16) GNPDE_SD(1, 16);
    else if (GL == 32) GNPDE_SD(1, 32);
    else GNPDE_SD(1, 64);
  }
#undef GNPDE_SD
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_softmax_backward_f32(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, int heads,
                               const float* att, const float* g, float* gs, void* stream) {
  GNPDE_REQUIRE(R >= 1 && nnz >= 0 && heads >= 1, GNPDE_EINVAL, "softmax_backward: bad sizes");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowptr && perm && att && g && gs, GNPDE_EINVAL, "softmax_backward: NULL pointer");
  softmax_backward_kernel<<<grid_n(R * kWave), kBlock, 0, as_stream(stream)>>>(rowptr, perm, R, heads, att, g, gs);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_segment_sum_f64(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, int heads,
                          const float* vals, double* out, void* stream) {
  GNPDE_REQUIRE(R >= 1 && nnz >= 0 && heads >= 1, GNPDE_EINVAL, "segment_sum: bad sizes");
  GNPDE_REQUIRE(rowptr && out && (nnz == 0 || (perm && vals)), GNPDE_EINVAL, "segment_sum: NULL pointer");
  segment_sum_kernel<<<grid_n(R * kWave), kBlock, 0, as_stream(stream)>>>(rowptr, perm, R, heads, vals, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

size_t gnpde_wcolsum_workspace_bytes(int64_t B, int64_t N, int64_t C, int heads) {
  int rpt, ntiles;
  wcolsum_geometry(B, N, &rpt, &ntiles);
  return sizeof(double) * (size_t)(B * heads * ntiles * (C + 1)) + 256;
}

int gnpde_wcolsum_f64(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const double* w, int heads,
                      double* y, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(x && w && y && workspace, GNPDE_EINVAL, "wcolsum: NULL pointer");
  GNPDE_REQUIRE(B >= 1 && N >= 1 && C >= 1 && ldx >= C && heads >= 1 && B <= 65535 && heads <= 65535,
                GNPDE_EINVAL, "wcolsum: bad sizes");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_wcolsum_workspace_bytes(B, N, C, heads), GNPDE_EINVAL,
                "wcolsum: workspace too small");
  int rpt, ntiles;
  wcolsum_geometry(B, N, &rpt, &ntiles);
  const int tpr = pow2_ge((int)C, 256);
  const int rpb = kBlock / tpr;
  const size_t shm = sizeof(double) * (size_t)rpb * (C + 1);
  GNPDE_REQUIRE(shm <= 64 * 1024, GNPDE_EUNSUPPORTED, "wcolsum: C too large");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  wcolsum_partial_kernel<<<dim3((unsigned)ntiles, (unsigned)B, (unsigned)heads), kBlock, shm, s>>>(
      x, N, (int)C, ldx, w, heads, rpt, tpr, ntiles, part);
  GNPDE_LAUNCH_CHECK();
  wcolsum_tiles_kernel<<<dim3((unsigned)ceil_div(C + 1, kBlock), (unsigned)(B * heads)), kBlock, 0, s>>>(
      part, ntiles, (int)(C + 1), y);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_score_input_grad_f32(const double* gcs, const double* U, const int32_t* deg, const double* gxbar, int64_t B,
                               int64_t N, int64_t C, int heads, float* gx, int64_t ldgx, int accumulate,
                               void* stream) {
  GNPDE_REQUIRE(gcs && U && deg && gxbar && gx, GNPDE_EINVAL, "score_input_grad: NULL pointer");
  GNPDE_REQUIRE(B >= 1 && N >= 1 && C >= 1 && ldgx >= C && heads >= 1, GNPDE_EINVAL, "score_input_grad: bad sizes");
  score_input_grad_kernel<<<grid_n(B * N * C), kBlock, 0, as_stream(stream)>>>(gcs, U, deg, gxbar, N, B * N, (int)C,
                                                                               heads, gx, ldgx, accumulate);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_gather_head_f32(const float* w, int64_t nnz, int heads, int h, const int32_t* perm, float scale, float* out,
                          void* stream) {
  GNPDE_REQUIRE(heads >= 1 && h >= 0 && h < heads && nnz >= 0, GNPDE_EINVAL, "gather_head: bad head");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(w && perm && out, GNPDE_EINVAL, "gather_head: NULL pointer");
  gather_head_kernel<<<grid_n(nnz), 256, 0, as_stream(stream)>>>(w, nnz, heads, h, perm, scale, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
