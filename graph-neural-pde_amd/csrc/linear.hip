// linear.hip — the dense node projections of the attention RHS (Q and K of
// SpGraphTransAttentionLayer, function_transformer_attention.py:224-225) on the
// CDNA4 matrix cores.
//
// Default (K % 16 == 0, K <= 128): linear_split_kernel, the f32 product formed
// from exact three-piece bf16 splits of both operands on
// v_mfma_f32_32x32x16_bf16 (16x the f32 MFMA rate; f32-GEMM accuracy, see the
// comment above it).  G-arxiv Q|K (R = 169,343, K = 128, Nout = 64): 32.8 us
// against 42.2 us for the exact-f32 kernel below (profiles/r02b_*).
//
// Other shapes: exact-f32 v_mfma_f32_32x32x2_f32 (one f32 fma chain per output,
// same numerics as an fp32 GEMM with a different summation order).  Tile: one
// wavefront = 32 rows x 64 output columns (two 32x32 accumulators),
// 4 wavefronts per workgroup = 128 rows; blockIdx.y walks 64-column slices of
// the output.  The K (= C) reduction is split between the two lane halves of
// the MFMA: half h covers k in [h*Kh, h*Kh + Kh), Kh = ceil(K/2), so each lane
// streams a contiguous run of its own x row (16-byte loads when K % 8 == 0).
// W^T for the slice is staged once per workgroup in LDS as [k][64 columns].
#include <algorithm>
#include <cstdlib>

#include "common.hpp"

namespace gnpde {

typedef float f32x16 __attribute__((ext_vector_type(16)));

constexpr int kLinRowsPerWave = 32;
constexpr int kLinCols = 64;

constexpr int kLinChunk = 16;        // k-steps per half per prefetch chunk
constexpr int kLinLdsStride = kLinCols + 1;
constexpr int kLinStageCols = kLinCols / kWavesPerBlock;  // W^T columns staged per wavefront
constexpr int kOutOfRange = 0x7ffffff0;                    // buffer offset past any W (reads 0)

// x elements as fp32: fp32 storage, or bf16 storage widened exactly (a bf16 state's
// projection reads it directly: the same values, so the same products and bits as
// the projection of its fp32 copy)
template <class XT>
__device__ __forceinline__ float4 lin_load4(const XT* __restrict__ p) {
  if constexpr (sizeof(XT) == 4) {
    return *reinterpret_cast<const float4*>(p);
  } else {
    const u32x2 w = *reinterpret_cast<const u32x2*>(p);
    return make_float4(__uint_as_float(w.x << 16), __uint_as_float(w.x & 0xffff0000u), __uint_as_float(w.y << 16),
                       __uint_as_float(w.y & 0xffff0000u));
  }
}
template <class XT>
__device__ __forceinline__ float lin_load1(const XT* __restrict__ p) {
  if constexpr (sizeof(XT) == 4)
    return *p;
  else
    return __uint_as_float((uint32_t)(*reinterpret_cast<const uint16_t*>(p)) << 16);
}

// A chunk of kLinChunk k-steps of this lane's half row (zeros past Kh / K).
template <bool VEC4, class XT = float>
__device__ __forceinline__ void lin_load_chunk(const XT* __restrict__ xr, int kbase, int s0, int Kh, int K,
                                               float (&a)[kLinChunk]) {
  if constexpr (VEC4) {
#pragma unroll
    for (int i = 0; i < kLinChunk; i += 4) {
      if (s0 + i < Kh) {
        const float4 t = lin_load4<XT>(xr + kbase + s0 + i);
        a[i] = t.x; a[i + 1] = t.y; a[i + 2] = t.z; a[i + 3] = t.w;
      } else {
        a[i] = a[i + 1] = a[i + 2] = a[i + 3] = 0.f;
      }
    }
  } else {
#pragma unroll
    for (int i = 0; i < kLinChunk; ++i) {
      const int k = kbase + s0 + i;
      a[i] = (s0 + i < Kh && k < K) ? lin_load1<XT>(xr + k) : 0.f;
    }
  }
}

// Stage W^T for the 64-column slice at col0 into LDS [2*Khp][65]: wave wv
// fills columns j = wv + 4*jj, lanes walk the k rows (coalesced along k).
// Buffer loads with 32-bit offsets: a padding element (k past the half, n past
// Nout) gets an out-of-range offset and reads 0, so all kLinStageCols loads
// issue back to back with no branch or 64-bit select.
__device__ __forceinline__ void lin_stage_wt(const float* __restrict__ W, int K, int Nout, int Kh, int Khp, int col0,
                                             int lane, int wv, float* __restrict__ wt) {
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(W), 0, Nout * K * (int)sizeof(float), 0x00020000);
  for (int kr = lane; kr < 2 * Khp; kr += kWave) {
    const int hh = kr >= Khp ? 1 : 0;
    const int sidx = kr - hh * Khp;
    const int k = hh * Kh + sidx;
    const bool kok = sidx < Kh && k < K;
    float val[kLinStageCols];
#pragma unroll
    for (int jj = 0; jj < kLinStageCols; ++jj) {
      const int n = col0 + wv + kWavesPerBlock * jj;
      const int off = (kok && n < Nout) ? (n * K + k) * (int)sizeof(float) : kOutOfRange;
      val[jj] = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(wr, off, 0, 0));
    }
#pragma unroll
    for (int jj = 0; jj < kLinStageCols; ++jj) wt[kr * kLinLdsStride + wv + kWavesPerBlock * jj] = val[jj];
  }
}

// K split between the MFMA lane halves: half h covers k = h*Kh + s, s < Kh.
// The LDS image of W^T has Khp = roundup(Kh, kLinChunk) rows per half (zero
// padded), so the MFMA loop runs whole chunks with no per-step guard.
template <bool VEC4, class XT = float>
__global__ __launch_bounds__(256) void linear_mfma_kernel(const XT* __restrict__ x, int R, int K, int64_t ldx,
                                                           const float* __restrict__ W,
                                                           const float* __restrict__ bias, int Nout, int split,
                                                           float* __restrict__ out_a, int64_t lda,
                                                           float* __restrict__ out_b, int64_t ldb) {
  extern __shared__ __attribute__((aligned(16))) float wt[];  // [2*Khp][65]
  const int Kh = (K + 1) >> 1;
  const int Khp = (Kh + kLinChunk - 1) / kLinChunk * kLinChunk;
  const int col0 = blockIdx.y * kLinCols;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int row0 = (blockIdx.x * kWavesPerBlock + wv) * kLinRowsPerWave;
  const bool wave_live = row0 < R;  // no early return: every wave takes part in the staging barrier
  const int my_row = min(row0 + r32, R - 1);
  const XT* __restrict__ xr = x + (int64_t)my_row * ldx;
  const int kbase = h * Kh;

  // this wave's first chunk of x goes out before the W^T staging
  float a_cur[kLinChunk], a_nxt[kLinChunk];
  lin_load_chunk<VEC4, XT>(xr, kbase, 0, Kh, K, a_cur);

  lin_stage_wt(W, K, Nout, Kh, Khp, col0, lane, wv, wt);
  __syncthreads();
  // Explicit: the loop head then sees no pending load, so the compiler's merge
  // there does not make every chunk wait for the next chunk's prefetch.
  __builtin_amdgcn_s_waitcnt(kWaitVm0);
  if (!wave_live) return;

  const float* __restrict__ wbase = wt + h * Khp * kLinLdsStride;
  f32x16 acc0 = {0}, acc1 = {0};
  for (int s0 = 0; s0 < Khp; s0 += kLinChunk) {
    if (s0 + kLinChunk < Khp) lin_load_chunk<VEC4, XT>(xr, kbase, s0 + kLinChunk, Kh, K, a_nxt);
    float b0[kLinChunk], b1[kLinChunk];
#pragma unroll
    for (int i = 0; i < kLinChunk; ++i) {
      const float* wrow = wbase + (s0 + i) * kLinLdsStride;
      b0[i] = wrow[r32];
      b1[i] = wrow[32 + r32];
    }
#pragma unroll
    for (int i = 0; i < kLinChunk; ++i) {
      acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[i], b0[i], acc0, 0, 0, 0);
      acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a_cur[i], b1[i], acc1, 0, 0, 0);
    }
#pragma unroll
    for (int i = 0; i < kLinChunk; ++i) a_cur[i] = a_nxt[i];
  }

  // Epilogue.  C/D layout (32x32): col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5).
  // Each lane owns one column per tile: its bias, destination (out_a or
  // out_b) and stride are fixed up front; a whole in-range tile stores with
  // no branch (a conditional store would make every later wait drain vmcnt,
  // stores included, serialising them).
  float bv[2];
  float* dst[2];
  int64_t ld[2];
#pragma unroll
  for (int tile = 0; tile < 2; ++tile) {
    const int n = col0 + tile * 32 + r32;
    const int nc = n < Nout ? n : 0;
    const float bb = bias ? bias[nc] : 0.f;
    bv[tile] = n < Nout ? bb : 0.f;
    const bool to_a = n < split;
    dst[tile] = to_a ? out_a + nc : out_b + (nc - split);
    ld[tile] = to_a ? lda : ldb;
  }
  const bool full = row0 + kLinRowsPerWave <= R && col0 + kLinCols <= Nout;
  if (full) {
#pragma unroll
    for (int reg = 0; reg < 16; ++reg) {
      const int row = row0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
      dst[0][(int64_t)row * ld[0]] = acc0[reg] + bv[0];
      dst[1][(int64_t)row * ld[1]] = acc1[reg] + bv[1];
    }
  } else {
#pragma unroll
    for (int tile = 0; tile < 2; ++tile) {
      const int n = col0 + tile * 32 + r32;
      if (n >= Nout) continue;
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = row0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        if (row < R) dst[tile][(int64_t)row * ld[tile]] = (tile == 0 ? acc0[reg] : acc1[reg]) + bv[tile];
      }
    }
  }
}


// Persistent variant for K <= 2*16*NCH, K % 8 == 0 (the usual attention widths): each
// workgroup stages its W^T slice ONCE and its wavefronts walk 32-row tiles
// (tile, tile + 4*gridDim.x, ...).  x of the current tile sits in registers
// (NCH*16 values per lane); as soon as chunk c has gone through the MFMAs its
// registers are reloaded with chunk c of the NEXT tile, so every load has
// (NCH - 1) chunks of matrix work to arrive in, with one x buffer.
template <bool VEC4, int NCH, class XT = float>
__global__ __launch_bounds__(256, 2) void linear_mfma_tiles_kernel(const XT* __restrict__ x, int R, int K,
                                                                    int64_t ldx, const float* __restrict__ W,
                                                                    const float* __restrict__ bias, int Nout,
                                                                    int split, float* __restrict__ out_a,
                                                                    int64_t lda, float* __restrict__ out_b,
                                                                    int64_t ldb) {
  constexpr int KS = NCH * kLinChunk;  // k-steps per half (Khp)
  extern __shared__ __attribute__((aligned(16))) float wt[];  // [2*KS][65]
  const int Kh = (K + 1) >> 1;
  const int col0 = blockIdx.y * kLinCols;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int kbase = h * Kh;
  const int ntiles = (R + kLinRowsPerWave - 1) / kLinRowsPerWave;
  const int step = gridDim.x * kWavesPerBlock;
  int tile = blockIdx.x * kWavesPerBlock + wv;

  // the wave's first tile goes out before the W^T staging
  float a[NCH][kLinChunk];
  {
    const XT* __restrict__ xr = x + (int64_t)min(min(tile, ntiles - 1) * kLinRowsPerWave + r32, R - 1) * ldx;
#pragma unroll
    for (int c = 0; c < NCH; ++c) lin_load_chunk<VEC4, XT>(xr, kbase, c * kLinChunk, Kh, K, a[c]);
  }
  lin_stage_wt(W, K, Nout, Kh, KS, col0, lane, wv, wt);
  __syncthreads();
  if (tile >= ntiles) return;

  // per-lane epilogue constants (one output column per accumulator tile)
  float bv[2];
  float* dst[2];
  int64_t ld[2];
#pragma unroll
  for (int tt = 0; tt < 2; ++tt) {
    const int n = col0 + tt * 32 + r32;
    const int nc = n < Nout ? n : 0;
    const float bb = bias ? bias[nc] : 0.f;
    bv[tt] = n < Nout ? bb : 0.f;
    const bool to_a = n < split;
    dst[tt] = to_a ? out_a + nc : out_b + (nc - split);
    ld[tt] = to_a ? lda : ldb;
  }
  const bool cols_full = col0 + kLinCols <= Nout;
  const float* __restrict__ wbase = wt + h * KS * kLinLdsStride;

  for (; tile < ntiles; tile += step) {
    // next tile (clamped: the last iteration re-reads a valid row, no branch)
    const int nt = min(tile + step, ntiles - 1);
    const XT* __restrict__ xn = x + (int64_t)min(nt * kLinRowsPerWave + r32, R - 1) * ldx;
    f32x16 acc0 = {0}, acc1 = {0};
#pragma unroll
    for (int c = 0; c < NCH; ++c) {
      float b0[kLinChunk], b1[kLinChunk];
#pragma unroll
      for (int i = 0; i < kLinChunk; ++i) {
        const float* wrow = wbase + (c * kLinChunk + i) * kLinLdsStride;
        b0[i] = wrow[r32];
        b1[i] = wrow[32 + r32];
      }
#pragma unroll
      for (int i = 0; i < kLinChunk; ++i) {
        acc0 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][i], b0[i], acc0, 0, 0, 0);
        acc1 = __builtin_amdgcn_mfma_f32_32x32x2f32(a[c][i], b1[i], acc1, 0, 0, 0);
      }
      lin_load_chunk<VEC4, XT>(xn, kbase, c * kLinChunk, Kh, K, a[c]);
      // keep chunks in program order: hoisting later chunks' LDS reads (or the
      // next tile's loads into fresh registers) would spill
      __builtin_amdgcn_sched_barrier(0);
    }
    // C/D layout (32x32): col = lane&31, row = (reg&3) + 8*(reg>>2) + 4*(lane>>5)
    const int row0 = tile * kLinRowsPerWave;
    if (row0 + kLinRowsPerWave <= R && cols_full) {
#pragma unroll
      for (int reg = 0; reg < 16; ++reg) {
        const int row = row0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
        dst[0][(int64_t)row * ld[0]] = acc0[reg] + bv[0];
        dst[1][(int64_t)row * ld[1]] = acc1[reg] + bv[1];
      }
    } else {
#pragma unroll
      for (int tt = 0; tt < 2; ++tt) {
        const int n = col0 + tt * 32 + r32;
        if (n >= Nout) continue;
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int row = row0 + (reg & 3) + 8 * (reg >> 2) + 4 * h;
          if (row < R) dst[tt][(int64_t)row * ld[tt]] = (tt == 0 ? acc0[reg] : acc1[reg]) + bv[tt];
        }
      }
    }
  }
}

// ------------------------------------------------------------------ split-bf16 projection
// The same product on the bf16 matrix cores, which run 16x the f32 MFMA rate:
// every f32 operand is split EXACTLY into three bf16 pieces, v = v0 + v1 + v2
// (v0 = RNE(v), v1 = RNE(v - v0), v2 = v - v0 - v1: each residual keeps at most
// 16, then 8 significant bits), and the six products whose magnitude is above
// 2^-24 of the leading one (x0w0, x0w1, x1w0, x0w2, x1w1, x2w0) are summed by
// v_mfma_f32_32x32x16_bf16 in f32.  The dropped ones (x1w2, x2w1, x2w2) are
// below 2^-24 |x||w|: f32-GEMM accuracy at 6/16 of the f32 MFMA cost, so the
// kernel is bound by its x stream instead of the matrix cores.
//
// Lane l = r + 32h of a wave owns row r of a 32-row tile and the K/2 contiguous
// columns [h*K/2, (h+1)*K/2) of it (one 16-byte load stream per lane); MFMA
// step s takes its 8 columns h*K/2 + 8s .. +7, i.e. the k index of the
// operand layout (8h + j) is permuted, identically for A (x) and B (W).  The
// B fragments of the 64-column slice — 2 tiles x 3 pieces x K/16 steps — are
// split once per workgroup into LDS in lane order (ds_read_b128,
// conflict-free).  Persistent waves walk tiles; as soon as step s has been
// split, its registers are refilled with step s of the next tile.
typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef uint32_t u32x4_t __attribute__((ext_vector_type(4)));

// one v_cvt_pk_bf16_f32 (RNE) per pair; the pair's f32 values of the pieces
// are the dword's halves moved to the high bits (shift / mask), the residuals
// one packed subtraction
__device__ __forceinline__ void split_pair(f32x2_t v, uint32_t& p0, uint32_t& p1, uint32_t& p2) {
  auto widen = [](uint32_t p) {
    const f32x2_t w = {__uint_as_float(p << 16), __uint_as_float(p & 0xffff0000u)};
    return w;
  };
  p0 = __builtin_bit_cast(uint32_t, __builtin_convertvector(v, bf16x2_t));
  const f32x2_t r1 = v - widen(p0);
  p1 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r1, bf16x2_t));
  const f32x2_t r2 = r1 - widen(p1);
  p2 = __builtin_bit_cast(uint32_t, __builtin_convertvector(r2, bf16x2_t));
}

__device__ __forceinline__ void split3(const float4& lo, const float4& hi, bf16x8_t& p0, bf16x8_t& p1,
                                       bf16x8_t& p2) {
  uint32_t a0, a1, a2, a3, b0, b1, b2, b3, c0, c1, c2, c3;
  const f32x2_t v0 = {lo.x, lo.y}, v1 = {lo.z, lo.w}, v2 = {hi.x, hi.y}, v3 = {hi.z, hi.w};
  split_pair(v0, a0, b0, c0);
  split_pair(v1, a1, b1, c1);
  split_pair(v2, a2, b2, c2);
  split_pair(v3, a3, b3, c3);
  const u32x4_t a = {a0, a1, a2, a3}, b = {b0, b1, b2, b3}, c = {c0, c1, c2, c3};
  p0 = __builtin_bit_cast(bf16x8_t, a);
  p1 = __builtin_bit_cast(bf16x8_t, b);
  p2 = __builtin_bit_cast(bf16x8_t, c);
}

// The product is formed transposed, D = W x^T (W fragments as the A operand,
// x as B), so that a lane ends with ITS row's outputs: 32 output columns of
// tile t in 4 runs of 4 (rows (reg&3) + 8*(reg>>2) + 4h of the C layout), i.e.
// four 16-byte stores per tile.  Stores are raw buffer stores with
// out-of-range offsets dropped (no branch: every path has the same vmcnt
// count, so the wait for a step's refill does not wait for the stores).
// VST: float4 stores (split % 32 == 0 or no second output, Nout % 4 == 0,
// 16-byte aligned outputs and strides); otherwise one store per element into
// both outputs, the one that does not own the column dropped.
template <int KS, bool VST, class XT = float>
__global__ __launch_bounds__(256, 2) void linear_split_kernel(const XT* __restrict__ x, int R, int64_t ldx,
                                                               const float* __restrict__ W,
                                                               const float* __restrict__ bias, int Nout, int split,
                                                               float* __restrict__ out_a, int64_t lda,
                                                               float* __restrict__ out_b, int64_t ldb) {
  constexpr int K = 16 * KS, KH = 8 * KS;
  extern __shared__ __attribute__((aligned(16))) bf16x8_t wfrag[];  // [tile 2][piece 3][step KS][lane 64] | bias[64]
  float* __restrict__ bl = reinterpret_cast<float*>(wfrag + 2 * 3 * KS * kWave);
  const int col0 = blockIdx.y * kLinCols;
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int r32 = lane & 31, h = lane >> 5;
  const int ntiles = (R + kLinRowsPerWave - 1) / kLinRowsPerWave;
  const int step = gridDim.x * kWavesPerBlock;
  int tile = blockIdx.x * kWavesPerBlock + wv;

  // the wave's first tile goes out before the W staging
  float4 xa[2 * KS];
  {
    const XT* __restrict__ xr =
        x + (int64_t)min(min(tile, ntiles - 1) * kLinRowsPerWave + r32, R - 1) * ldx + h * KH;
#pragma unroll
    for (int i = 0; i < 2 * KS; ++i) xa[i] = lin_load4<XT>(xr + 4 * i);
  }
  for (int e = threadIdx.x; e < 2 * KS * kWave; e += kBlock) {
    const int t = e / (KS * kWave), s = (e / kWave) % KS, l = e % kWave;
    const int n = col0 + 32 * t + (l & 31);
    float4 lo = make_float4(0.f, 0.f, 0.f, 0.f), hi = lo;
    if (n < Nout) {
      const float* wr = W + (int64_t)n * K + (l >> 5) * KH + 8 * s;
      lo = *reinterpret_cast<const float4*>(wr);
      hi = *reinterpret_cast<const float4*>(wr + 4);
    }
    bf16x8_t p0, p1, p2;
    split3(lo, hi, p0, p1, p2);
    wfrag[((t * 3 + 0) * KS + s) * kWave + l] = p0;
    wfrag[((t * 3 + 1) * KS + s) * kWave + l] = p1;
    wfrag[((t * 3 + 2) * KS + s) * kWave + l] = p2;
  }
  if (threadIdx.x < kLinCols) {
    const int n = col0 + threadIdx.x;
    bl[threadIdx.x] = (bias && n < Nout) ? bias[n] : 0.f;
  }
  __syncthreads();
  if (tile >= ntiles) return;

  const __amdgpu_buffer_rsrc_t ra = buf_rsrc(out_a);
  const __amdgpu_buffer_rsrc_t rb = buf_rsrc(out_b ? out_b : out_a);

  for (; tile < ntiles; tile += step) {
    const int nt = min(tile + step, ntiles - 1);  // clamped: the last pass re-reads a valid row
    const XT* __restrict__ xn = x + (int64_t)min(nt * kLinRowsPerWave + r32, R - 1) * ldx + h * KH;
    f32x16 acc[2] = {{0}, {0}};
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      bf16x8_t a0, a1, a2;
      split3(xa[2 * s], xa[2 * s + 1], a0, a1, a2);
      // refill four steps at a time: the lane's 128-byte line of the next tile
      // is then read by eight back-to-back loads (spread over four steps, its
      // line left the 32 KB L1 between them and was fetched again from L2)
      if (s % 4 == 3 || s == KS - 1) {
#pragma unroll
        for (int s2 = s - s % 4; s2 <= s; ++s2) {
          xa[2 * s2] = lin_load4<XT>(xn + 8 * s2);
          xa[2 * s2 + 1] = lin_load4<XT>(xn + 8 * s2 + 4);
        }
      }
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const bf16x8_t w0 = wfrag[((t * 3 + 0) * KS + s) * kWave + lane];
        const bf16x8_t w1 = wfrag[((t * 3 + 1) * KS + s) * kWave + lane];
        const bf16x8_t w2 = wfrag[((t * 3 + 2) * KS + s) * kWave + lane];
        // smallest products first
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a2, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, a1, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w2, a0, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a1, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w1, a0, acc[t], 0, 0, 0);
        acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(w0, a0, acc[t], 0, 0, 0);
      }
      // keep step s+1's refill behind step s+1's split: hoisted above it, the
      // refill needs fresh registers and the loop head then copies them back
      // after waiting for almost every load of the next tile
      asm volatile("" ::: "memory");
      __builtin_amdgcn_sched_barrier(0);
    }
    // D = W x^T in the C layout: lane column = x row r32, register 4g + i = output
    // column 8g + 4h + i of tile t
    const int row = tile * kLinRowsPerWave + r32;
    const bool row_ok = row < R;
#pragma unroll
    for (int t = 0; t < 2; ++t) {
      const int n0 = col0 + 32 * t;  // wave-uniform
      if constexpr (VST) {
        const bool to_a = n0 < split;
        const int64_t ld = to_a ? lda : ldb;
        const int nb = to_a ? n0 : n0 - split;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          const int c = 8 * g + 4 * h;
          const float4 b4 = *reinterpret_cast<const float4*>(bl + 32 * t + c);
          const u32x4_t d = {__float_as_uint(acc[t][4 * g] + b4.x), __float_as_uint(acc[t][4 * g + 1] + b4.y),
                             __float_as_uint(acc[t][4 * g + 2] + b4.z), __float_as_uint(acc[t][4 * g + 3] + b4.w)};
          const uint32_t off = (row_ok && n0 + c < Nout) ? (uint32_t)(((int64_t)row * ld + nb + c) * 4) : kBufNone;
          __builtin_amdgcn_raw_buffer_store_b128(d, to_a ? ra : rb, off, 0, 0);
        }
      } else {
#pragma unroll
        for (int reg = 0; reg < 16; ++reg) {
          const int n = n0 + 8 * (reg >> 2) + 4 * h + (reg & 3);
          const float v = acc[t][reg] + bl[n - col0];
          const bool ok = row_ok && n < Nout;
          const uint32_t oa = (ok && n < split) ? (uint32_t)(((int64_t)row * lda + n) * 4) : kBufNone;
          const uint32_t ob = (ok && n >= split) ? (uint32_t)(((int64_t)row * ldb + n - split) * 4) : kBufNone;
          buf_store_f32(ra, oa, v);
          buf_store_f32(rb, ob, v);
        }
      }
    }
  }
}


}  // namespace gnpde

using namespace gnpde;

// Measured and dropped (round 3): x tiles moved by the DMA path into LDS
// (global_load_lds_dwordx4, two 16-KB buffers per wave, rows rotated by one 16-B
// slot per row against bank conflicts, 3 waves per CU to fit 48 KB of W fragments +
// 96 KB of tiles): 39.7 us against 33 us — one wave per SIMD at most cannot hide
// the next tile's latency behind one tile of matrix work.
// Experiment builds only (GNPDE_EXPERIMENTS): GNPDE_LINEAR=1 forces the
// per-tile (non-persistent) exact-f32 kernel, =2 the persistent exact-f32 one
// (default: the split-bf16 kernel where K % 16 == 0 and K <= 128).  Measured
// and dropped: 16-row tiles on 16x16x32 with a three-deep register ring of x
// tiles (31.7-32.3 us), splitting the whole tile before refilling (1 wave per
// SIMD, 32-38 us), refilling per step instead of per 128-byte line (32 us).
static int linear_variant() {
  if constexpr (!GNPDE_EXPERIMENTS) return 0;
  static const int v = [] {
    const char* e = std::getenv("GNPDE_LINEAR");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

// Experiment builds only: GNPDE_LIN_WAVES = wavefronts of the
// persistent projection grid (default 2048).
static int64_t linear_waves() {
  if constexpr (!GNPDE_EXPERIMENTS) return 2048;
  static const int64_t v = [] {
    const char* e = std::getenv("GNPDE_LIN_WAVES");
    return e ? std::max<int64_t>(4, std::atoll(e)) : (int64_t)2048;
  }();
  return v;
}

template <class XT>
static int linear_impl(const XT* x, int64_t R, int64_t K, int64_t ldx, const float* W, const float* bias, int64_t Nout,
                       int64_t split, float* out_a, int64_t lda, float* out_b, int64_t ldb, void* stream) {
  GNPDE_REQUIRE(x && W && out_a, GNPDE_EINVAL, "linear: NULL pointer");
  GNPDE_REQUIRE(R >= 0 && R < INT32_MAX && K >= 1 && ldx >= K && Nout >= 1, GNPDE_EINVAL, "linear: bad sizes");
  GNPDE_REQUIRE(split >= 0 && split <= Nout, GNPDE_EINVAL, "linear: bad split");
  GNPDE_REQUIRE(Nout * K * (int64_t)sizeof(float) < kOutOfRange, GNPDE_EUNSUPPORTED, "linear: W larger than 2 GB");
  GNPDE_REQUIRE(split == Nout || out_b != nullptr, GNPDE_EINVAL, "linear: out_b is NULL");
  GNPDE_REQUIRE(lda >= split && (split == Nout || ldb >= Nout - split), GNPDE_EINVAL, "linear: bad ld");
  const int64_t Kh = (K + 1) / 2;
  const int64_t Khp = (Kh + kLinChunk - 1) / kLinChunk * kLinChunk;
  const size_t shm = sizeof(float) * (size_t)(2 * Khp * kLinLdsStride);
  GNPDE_REQUIRE(shm <= 160 * 1024, GNPDE_EUNSUPPORTED, "linear: K=%lld too large for the LDS slice",
                (long long)K);
  if (R == 0) return GNPDE_OK;
  // fp32: 16-byte x loads; bf16: 8-byte loads of four elements
  const bool vec4 = (K % 8 == 0) && (ldx % 4 == 0) && (sizeof(XT) == 4 ? aligned16(x) : aligned8(x));
  hipStream_t s = as_stream(stream);
  const int nch = (int)(Khp / kLinChunk);
  if (vec4 && K % 16 == 0 && K <= 128 && aligned16(W) && linear_variant() == 0 &&
      R * std::max(lda, split == Nout ? lda : ldb) * (int64_t)sizeof(float) < (int64_t)kBufRecords) {
    // split-bf16 MFMA, persistent tiles (same wave budget as below)
    const int64_t ntiles = ceil_div(R, kLinRowsPerWave);
    const int64_t slices = ceil_div(Nout, kLinCols);
    const int64_t max_waves = std::max<int64_t>(kWavesPerBlock, linear_waves() / slices);
    const int64_t per_wave = ceil_div(ntiles, max_waves);
    const int64_t blocks = ceil_div(ceil_div(ntiles, per_wave), kWavesPerBlock);
    const dim3 gt((unsigned)blocks, (unsigned)slices);
    const size_t lds = sizeof(bf16x8_t) * 2 * 3 * (size_t)(K / 16) * kWave + sizeof(float) * kLinCols;
    const bool vst = (split % 32 == 0 || split == Nout) && Nout % 4 == 0 && lda % 4 == 0 && aligned16(out_a) &&
                     (split == Nout || (ldb % 4 == 0 && aligned16(out_b)));
#define GNPDE_LIN_S(KS)                                                                                         \
  do {                                                                                                          \
    if (vst)                                                                                                    \
      linear_split_kernel<KS, true, XT><<<gt, kBlock, lds, s>>>(x, (int)R, ldx, W, bias, (int)Nout, (int)split,     \
                                                            out_a, lda, out_b, ldb);                            \
    else                                                                                                        \
      linear_split_kernel<KS, false, XT><<<gt, kBlock, lds, s>>>(x, (int)R, ldx, W, bias, (int)Nout, (int)split,    \
                                                             out_a, lda, out_b, ldb);                           \
  } while (0)
    switch (K / 16) {
      case 1: GNPDE_LIN_S(1); break;
      case 2: GNPDE_LIN_S(2); break;
      case 3: GNPDE_LIN_S(3); break;
      case 4: GNPDE_LIN_S(4); break;
      case 5: GNPDE_LIN_S(5); break;
      case 6: GNPDE_LIN_S(6); break;
      case 7: GNPDE_LIN_S(7); break;
      default: GNPDE_LIN_S(8); break;
    }
#undef GNPDE_LIN_S
    GNPDE_LAUNCH_CHECK();
    return GNPDE_OK;
  }
  if (vec4 && nch <= 6 && linear_variant() != 1) {
    // persistent tiles: about 2 workgroups per CU, tiles spread evenly over the wavefronts
    const int64_t ntiles = ceil_div(R, kLinRowsPerWave);
    const int64_t slices = ceil_div(Nout, kLinCols);
    const int64_t max_waves = std::max<int64_t>(kWavesPerBlock, linear_waves() / slices);
    const int64_t per_wave = ceil_div(ntiles, max_waves);
    const int64_t blocks = ceil_div(ceil_div(ntiles, per_wave), kWavesPerBlock);
    const dim3 gt((unsigned)blocks, (unsigned)slices);
#define GNPDE_LIN_T(N) \
  linear_mfma_tiles_kernel<true, N, XT><<<gt, kBlock, shm, s>>>(x, (int)R, (int)K, ldx, W, bias, (int)Nout, (int)split, \
                                                             out_a, lda, out_b, ldb)
    switch (nch) {
      case 1: GNPDE_LIN_T(1); break;
      case 2: GNPDE_LIN_T(2); break;
      case 3: GNPDE_LIN_T(3); break;
      case 4: GNPDE_LIN_T(4); break;
      case 5: GNPDE_LIN_T(5); break;
      default: GNPDE_LIN_T(6); break;
    }
#undef GNPDE_LIN_T
    GNPDE_LAUNCH_CHECK();
    return GNPDE_OK;
  }
  const dim3 grid((unsigned)ceil_div(R, kWavesPerBlock * kLinRowsPerWave), (unsigned)ceil_div(Nout, kLinCols));
  if (vec4)
    linear_mfma_kernel<true, XT><<<grid, kBlock, shm, s>>>(x, (int)R, (int)K, ldx, W, bias, (int)Nout, (int)split, out_a,
                                                      lda, out_b, ldb);
  else
    linear_mfma_kernel<false, XT><<<grid, kBlock, shm, s>>>(x, (int)R, (int)K, ldx, W, bias, (int)Nout, (int)split, out_a,
                                                       lda, out_b, ldb);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" int gnpde_linear_f32(const float* x, int64_t R, int64_t K, int64_t ldx, const float* W, const float* bias,
                                int64_t Nout, int64_t split, float* out_a, int64_t lda, float* out_b, int64_t ldb,
                                void* stream) {
  return linear_impl<float>(x, R, K, ldx, W, bias, Nout, split, out_a, lda, out_b, ldb, stream);
}

extern "C" int gnpde_linear_bf16(const void* x, int64_t R, int64_t K, int64_t ldx, const float* W, const float* bias,
                                 int64_t Nout, int64_t split, float* out_a, int64_t lda, float* out_b, int64_t ldb,
                                 void* stream) {
  return linear_impl<bf16>(static_cast<const bf16*>(x), R, K, ldx, W, bias, Nout, split, out_a, lda, out_b, ldb,
                           stream);
}
