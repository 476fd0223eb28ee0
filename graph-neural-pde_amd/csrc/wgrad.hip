// wgrad.hip — the weight gradient of the attention projections on the matrix
// cores: gW[m, k] = sum_r gy[r, m] x[r, k] (gy = dL/d[q | k] [R, M], x the node
// state [R, K]), the backward of nn.Linear's weight for SpGraphTransAttentionLayer's
// Q and K (function_transformer_attention.py:224-225), which torch autograd forms
// with a library GEMM.  The reduction runs over the R rows.
//
// v_mfma_f32_32x32x2_f32 (exact fp32 products, fp32 accumulation): a step takes
// two rows r0, r0 + 1; the A operand of lane l is gy[r0 + l/32][m0 + l%32] and the
// B operand x[r0 + l/32][k0 + l%32], so both are plain coalesced 128-byte half-row
// loads — the row dimension, the GEMM's reduction dimension, needs no transpose.
// A wavefront owns TM x TK output tiles of 32 x 32 (accumulators in AGPRs) and a
// contiguous range of row pairs; its partial tiles go to the workspace and
// wgrad_reduce_kernel sums the wavefronts' partials in wave order (fixed order:
// deterministic, no float atomics).
#include "common.hpp"

namespace gnpde {

typedef float f32x16w __attribute__((ext_vector_type(16)));
constexpr int kWgWaves = 512;  // most row ranges (wavefronts) per tile group
constexpr int64_t kWgRowsMin = 128;                 // fewest rows a range is given
constexpr int64_t kWgWorkspaceMax = 64ll << 20;     // partials budget (bytes) when M x K is large

// Row ranges for R rows and an M x K result: enough wavefronts to fill the chip on a
// large R, no more than R / kWgRowsMin, and no more partial tiles than kWgWorkspaceMax
// holds (a fixed 512 cost 128 MiB of scratch and traffic at M = K = 256);
// a multiple of the waves per workgroup.
static int64_t wgrad_waves(int64_t R, int64_t M, int64_t K) {
  int64_t nw = std::min<int64_t>(kWgWaves, std::max<int64_t>(1, ceil_div(R, kWgRowsMin)));
  nw = std::min<int64_t>(nw, std::max<int64_t>(1, kWgWorkspaceMax / (M * K * (int64_t)sizeof(float))));
  return ceil_div(nw, kWavesPerBlock) * kWavesPerBlock;
}

template <int TM, int TK>
__global__ __launch_bounds__(256) void wgrad_kernel(const float* __restrict__ gy, int64_t R, int M, int64_t ldg,
                                                     const float* __restrict__ x, int K, int64_t ldx,
                                                     float* __restrict__ part, int64_t rows_per_wave, int tgk) {
  const int lane = threadIdx.x & 63;
  const int w = blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);  // row-range index
  const int tg = blockIdx.y;                                        // tile group
  const int m0 = (tg / tgk) * TM * 32, k0 = (tg % tgk) * TK * 32;
  const int half = lane >> 5, c = lane & 31;
  const int64_t r_begin = (int64_t)w * rows_per_wave, r_end = min(R, r_begin + rows_per_wave);
  f32x16w acc[TM][TK];
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) acc[i][j] = f32x16w{0};
  bool mok[TM], kok[TK];
#pragma unroll
  for (int i = 0; i < TM; ++i) mok[i] = m0 + i * 32 + c < M;
#pragma unroll
  for (int j = 0; j < TK; ++j) kok[j] = k0 + j * 32 + c < K;
  constexpr int P = 4;  // row pairs in flight
  for (int64_t r0 = r_begin; r0 < r_end; r0 += 2 * P) {
    float a[P][TM], b[P][TK];
#pragma unroll
    for (int p = 0; p < P; ++p) {
      const int64_t r = r0 + 2 * p + half;
      const bool rok = r < r_end;
#pragma unroll
      for (int i = 0; i < TM; ++i) a[p][i] = (rok && mok[i]) ? gy[r * ldg + m0 + i * 32 + c] : 0.f;
#pragma unroll
      for (int j = 0; j < TK; ++j) b[p][j] = (rok && kok[j]) ? x[r * ldx + k0 + j * 32 + c] : 0.f;
    }
#pragma unroll
    for (int p = 0; p < P; ++p)
#pragma unroll
      for (int i = 0; i < TM; ++i)
#pragma unroll
        for (int j = 0; j < TK; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a[p][i], b[p][j], acc[i][j], 0, 0, 0);
  }
  // C/D layout (32x32): column = lane & 31 (k), row = (reg & 3) + 8 * (reg >> 2) + 4 * (lane >> 5) (m)
  float* __restrict__ pw = part + (int64_t)w * M * K;
#pragma unroll
  for (int i = 0; i < TM; ++i)
#pragma unroll
    for (int j = 0; j < TK; ++j) {
      const int k = k0 + j * 32 + c;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int m = m0 + i * 32 + (reg & 3) + 8 * (reg >> 2) + 4 * half;
        if (m < M && k < K) pw[(int64_t)m * K + k] = acc[i][j][reg];
      }
    }
}

// out[m, k] = sum over the nw wavefronts' partials, in wave order
__global__ __launch_bounds__(256) void wgrad_reduce_kernel(const float* __restrict__ part, int nw, int64_t MK,
                                                            int K, float* __restrict__ out, int64_t ldo) {
  const int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= MK) return;
  float s = 0.f;
  for (int w = 0; w < nw; ++w) s += part[(int64_t)w * MK + e];
  out[(e / K) * ldo + e % K] = s;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

size_t gnpde_linear_wgrad_workspace_bytes(int64_t R, int64_t M, int64_t K) {
  if (R < 0 || M < 1 || K < 1) return 0;
  return (size_t)wgrad_waves(R, M, K) * M * K * sizeof(float);
}

int gnpde_linear_wgrad_f32(const float* gy, int64_t R, int64_t M, int64_t ldg, const float* x, int64_t K, int64_t ldx,
                           float* gW, int64_t ldw, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(gW && (R == 0 || (gy && x)), GNPDE_EINVAL, "linear_wgrad: NULL pointer");
  GNPDE_REQUIRE(R >= 0 && M >= 1 && K >= 1 && ldg >= M && ldx >= K && ldw >= K && M <= 65536 && K <= 65536,
                GNPDE_EINVAL, "linear_wgrad: bad sizes");
  GNPDE_REQUIRE(workspace && workspace_bytes >= gnpde_linear_wgrad_workspace_bytes(R, M, K), GNPDE_EINVAL,
                "linear_wgrad: workspace smaller than gnpde_linear_wgrad_workspace_bytes");
  hipStream_t s = as_stream(stream);
  float* part = static_cast<float*>(workspace);
  const int MT = (int)ceil_div(M, 32), KT = (int)ceil_div(K, 32);
  const int TM = MT >= 2 ? 2 : 1;
  const int TK = KT >= 4 ? 4 : (KT >= 2 ? 2 : 1);
  const int tgm = (int)ceil_div(MT, TM), tgk = (int)ceil_div(KT, TK);
  // row pairs spread evenly over the wavefronts (an even count per wave keeps the pairs aligned)
  const int64_t nw = wgrad_waves(R, M, K);
  int64_t rpw = ceil_div(R, nw);
  rpw += rpw & 1;
  const dim3 grid((unsigned)(nw / kWavesPerBlock), (unsigned)(tgm * tgk));
#define GNPDE_WG(A, B)                                                                                         \
  wgrad_kernel<A, B><<<grid, kBlock, 0, s>>>(gy, R, (int)M, ldg, x, (int)K, ldx, part, std::max<int64_t>(rpw, 2), \
                                             tgk)
  if (TM == 2 && TK == 4) GNPDE_WG(2, 4);
  else if (TM == 2 && TK == 2) GNPDE_WG(2, 2);
  else if (TM == 2) GNPDE_WG(2, 1);
  else if (TK == 4) GNPDE_WG(1, 4);
  else if (TK == 2) GNPDE_WG(1, 2);
  else GNPDE_WG(1, 1);
#undef GNPDE_WG
  GNPDE_LAUNCH_CHECK();
  const int64_t MK = M * K;
  wgrad_reduce_kernel<<<(unsigned)ceil_div(MK, (int64_t)kBlock), kBlock, 0, s>>>(part, (int)nw, MK, (int)K, gW, ldw);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
