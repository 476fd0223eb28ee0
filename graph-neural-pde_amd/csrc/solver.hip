// solver.hip — fused Runge-Kutta stage combination: one streaming pass for
// y0 + dt * sum_j b_j k_j (torchdiffeq's rk4_alt_step_func / _runge_kutta_step
// do it with several elementwise torch kernels per stage); and the fp64 dot
// product of two fp32 tensors the parameter gradients of the RHS need
// (d alpha_train = sigma'(alpha) <gf, A x - x>, d beta_train = <gf, x0>).
#include "rhs_host.hpp"

namespace gnpde {

constexpr int kMaxStages = 8;

struct CombineArgs {
  const float* k[kMaxStages];
  float c[kMaxStages];
  int nk;
};

template <bool VEC4>
__global__ __launch_bounds__(256) void rk_combine_kernel(int64_t n, const float* __restrict__ y0, CombineArgs a,
                                                          float* __restrict__ out) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  if constexpr (VEC4) {
    const int64_t n4 = n >> 2;
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += stride) {
      float4 acc = y0 ? reinterpret_cast<const float4*>(y0)[i] : make_float4(0.f, 0.f, 0.f, 0.f);
      for (int j = 0; j < a.nk; ++j) {
        const float4 v = reinterpret_cast<const float4*>(a.k[j])[i];
        acc.x = fmaf(a.c[j], v.x, acc.x);
        acc.y = fmaf(a.c[j], v.y, acc.y);
        acc.z = fmaf(a.c[j], v.z, acc.z);
        acc.w = fmaf(a.c[j], v.w, acc.w);
      }
      reinterpret_cast<float4*>(out)[i] = acc;
    }
  } else {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
      float acc = y0 ? y0[i] : 0.f;
      for (int j = 0; j < a.nk; ++j) acc = fmaf(a.c[j], a.k[j][i], acc);
      out[i] = acc;
    }
  }
}

// <a, b> in fp64: a fixed grid of kDotBlocks blocks, each thread summing a fixed
// set of elements in order, a fixed tree per block, then one block summing the
// block partials in order — the same bits on every run (no float atomics).
constexpr int kDotBlocks = 1024;

__device__ __forceinline__ double block_sum_f64(double v, double* red) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v += __shfl_xor(v, o);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) red[wv] = v;
  __syncthreads();
  double t = 0.0;
  if (threadIdx.x == 0)
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) t += red[w];
  return t;  // thread 0 only
}

template <bool VEC4>
__global__ __launch_bounds__(256) void dot_partial_kernel(int64_t n, const float* __restrict__ a,
                                                           const float* __restrict__ b, double* __restrict__ part) {
  __shared__ double red[kBlock / kWave];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  if constexpr (VEC4) {
    const float4* a4 = reinterpret_cast<const float4*>(a);
    const float4* b4 = reinterpret_cast<const float4*>(b);
#pragma unroll 4
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < (n >> 2); i += stride) {
      const float4 u = a4[i], v = b4[i];
      acc = fma((double)u.x, (double)v.x, acc);
      acc = fma((double)u.y, (double)v.y, acc);
      acc = fma((double)u.z, (double)v.z, acc);
      acc = fma((double)u.w, (double)v.w, acc);
    }
  } else {
    for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride)
      acc = fma((double)a[i], (double)b[i], acc);
  }
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void dot_final_kernel(const double* __restrict__ part, int nb,
                                                         double* __restrict__ out) {
  __shared__ double red[kBlock / kWave];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) *out = t;
}

// sum of n doubles: the same fixed grid and per-block tree as dot_partial_kernel
__global__ __launch_bounds__(256) void sum_partial_kernel(int64_t n, const double* __restrict__ v,
                                                           double* __restrict__ part) {
  __shared__ double red[kBlock / kWave];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) acc += v[i];
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) part[blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void sum_final_kernel(const double* __restrict__ part, int nb, double* out,
                                                         int accumulate) {
  __shared__ double red[kBlock / kWave];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) *out = accumulate ? *out + t : t;
}

// Entry of a solve: dst[k] = src[order[k]] (and dst_copy[order[k]] = the same row)
// in 16-byte pieces, one thread per piece, consecutive threads along a row.
template <bool ORDER, bool COPY>
__global__ __launch_bounds__(256) void rows_copy_kernel(const uint4* __restrict__ src, int64_t rows, int64_t v4,
                                                         const int64_t* __restrict__ order, uint4* __restrict__ dst,
                                                         uint4* __restrict__ dst_copy) {
  const int64_t n = rows * v4;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    const int64_t k = i / v4, j = i - k * v4;
    const int64_t r = ORDER ? order[k] : k;
    const uint4 v = src[r * v4 + j];
    dst[i] = v;
    if constexpr (COPY) dst_copy[r * v4 + j] = v;
  }
}

// The stage epilogue as a pass of its own (gnpde_stage_apply_*): GL lanes per row
// (RPW = 64 / GL rows per wavefront), VEC elements per lane, column passes of
// GL*VEC.  Per element the same arithmetic, in the same order, as epi_finish
// (cb*base, the operands by fmaf in index order, then cf*f), so the pass and the
// fused epilogue give the same bits from the same f; the error rows summed over
// the row's lanes by the same xor tree.
// NKMAX / NOUT / ERR: the operands, outputs and error term an instantiation holds
// registers for (the plain combinations of the adaptive step — its first stage input,
// the dense output — take the lighter ones: more waves, more bytes in flight).
template <int VEC, int GL, class T, int NKMAX, int NOUT, bool ERR>
__global__ __launch_bounds__(256) void stage_apply_kernel(int64_t R, int C, int64_t ld, const T* __restrict__ f,
                                                           const T* __restrict__ x, gnpde_stage_epilogue_t st) {
  constexpr int RPW = kWave / GL;
  const int lane = threadIdx.x & 63;
  const int rs = lane / GL, gl = lane % GL;
  const int64_t row = ((int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * RPW + rs;
  const bool live = row < R;
  float dpart = 0.f;  // the error row's slice sums: fp32, as the fused epilogue (err_terms, epi_rowsums)
  for (int c0 = 0; c0 < C; c0 += GL * VEC) {
    const int cc = c0 + gl * VEC;
    if (!live || cc >= C) continue;
    const int64_t off = row * ld + cc;
    float fv[VEC], xv[VEC];
    if (f) {
      load_vec<VEC>(f + off, fv);
    } else {
#pragma unroll
      for (int t = 0; t < VEC; ++t) fv[t] = 0.f;
    }
    if (x) {
      load_vec<VEC>(x + off, xv);
    } else {
#pragma unroll
      for (int t = 0; t < VEC; ++t) xv[t] = 0.f;
    }
    if (st.f_lin != 0.f && x) {  // f = x + sc*f_lin*f, as the fused epilogue (ABI 5)
      const float cl = stage_scale(st) * st.f_lin;
#pragma unroll
      for (int t = 0; t < VEC; ++t) fv[t] = fmaf(cl, fv[t], xv[t]);
    }
    if (st.f_out) store_vec<VEC>(as_t<T>(st.f_out) + off, fv);
    float r[2][VEC], ev[VEC];
    Packed<VEC, T> y0v;
    wide_combine<VEC, T, NKMAX, NOUT, ERR>(st, off, fv, x ? reinterpret_cast<const float*>(x) : nullptr, xv, r, ev,
                                           &y0v);
    const int64_t oo = st.out_rows ? (int64_t)st.out_rows[row] * ld + cc : off;
#pragma unroll
    for (int i = 0; i < NOUT; ++i)
      if (i < st.n_out) store_vec<VEC>(as_t<T>(st.o[i].out) + oo, r[i]);
    if (ERR && st.err_rows) {
      float y1[VEC];
#pragma unroll
      for (int t = 0; t < VEC; ++t) y1[t] = st.err_y1 == 1 ? r[1][t] : (st.err_y1 == 0 ? r[0][t] : xv[t]);
      dpart += (float)err_terms<VEC, T>(st, off, ev, y1, &y0v);
    }
  }
  if (ERR && st.err_rows) {  // kernel-uniform
#pragma unroll
    for (int o = 1; o < GL; o <<= 1) dpart += __shfl_xor(dpart, o);
    if (live && gl == 0) st.err_rows[row] = (double)dpart;
  }
}

// ------------------------------------------------------------------ initial step
// torchdiffeq's _select_initial_step (misc.py, called by RKAdaptiveStepsizeODESolver
// ._before_integrate with order - 1; integrator._RKAdaptive._select_initial_step):
//   scale = atol + |y0| rtol,  d0 = rms(y0/scale),  d1 = rms(f0/scale)
//   h0 = 1e-6 if d0 < 1e-5 or d1 < 1e-5 else 0.01 d0/d1;  f1 = f(t0 + h0, y0 + h0 f0)
//   d2 = rms((f1 - f0)/scale)/h0
//   h1 = max(1e-6, 1e-3 h0) if d1 <= 1e-15 and d2 <= 1e-15 else (0.01/max(d1, d2))^(1/order)
//   first step = min(100 h0, h1)
// as two fixed-order reductions (no float atomics: the same bits every run) whose
// last block applies the scalar rules on the device, so the host reads the step
// once.  Elementwise arithmetic in fp32 as torch runs it on an fp32 state (the
// 0-d fp64 atol / rtol tensors do not promote it), squares summed in fp64.
template <class T, int VEC, int PHASE>
__global__ __launch_bounds__(256) void init_step_partial_kernel(int64_t n, const T* __restrict__ y0,
                                                                 const T* __restrict__ f0, const T* __restrict__ f1,
                                                                 float atol, float rtol, double* __restrict__ part) {
  __shared__ double red[kBlock / kWave];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double a0 = 0.0, a1 = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n / VEC; i += stride) {
    float y[VEC], f[VEC], g[VEC];
    load_vec<VEC>(y0 + i * VEC, y);
    if constexpr (PHASE != 2) load_vec<VEC>(f0 + i * VEC, f);
    if constexpr (PHASE >= 1) load_vec<VEC>(f1 + i * VEC, g);
#pragma unroll
    for (int t = 0; t < VEC; ++t) {
      const float sc = __fadd_rn(atol, __fmul_rn(fabsf(y[t]), rtol));  // no fma: torch rounds twice
      if constexpr (PHASE == 0) {
        const double q0 = (double)(y[t] / sc), q1 = (double)(f[t] / sc);
        a0 = fma(q0, q0, a0);
        a1 = fma(q1, q1, a1);
      } else if constexpr (PHASE == 1) {
        const double q = (double)((g[t] - f[t]) / sc);
        a0 = fma(q, q, a0);
      } else {  // PHASE 2: g = L f0 itself (gnpde_initial_step_lin_*)
        const double q = (double)(g[t] / sc);
        a0 = fma(q, q, a0);
      }
    }
  }
  const double t0 = block_sum_f64(a0, red);
  __syncthreads();
  const double t1 = PHASE == 0 ? block_sum_f64(a1, red) : 0.0;
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = t0;
    part[2 * blockIdx.x + 1] = t1;
  }
}

// h[0] = h0, h[1] = d1 (phase 0; hf = (float)h0, the probe's coefficient scale);
// h[2] = the first step (phase 1; DIVH: the sums are of (f1 - f0)/scale, divided by h0 —
// else of L f0 / scale, gnpde_initial_step_rows)
template <int PHASE, bool DIVH = true>
__global__ __launch_bounds__(256) void init_step_final_kernel(const double* __restrict__ part, int nb, double n,
                                                               double order, double* h, float* hf) {
  __shared__ double red[kBlock / kWave];
  double a0 = 0.0, a1 = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    a0 += part[2 * i];
    a1 += part[2 * i + 1];
  }
  const double s0 = block_sum_f64(a0, red);
  __syncthreads();
  const double s1 = block_sum_f64(a1, red);
  if (threadIdx.x != 0) return;
  if constexpr (PHASE == 0) {
    const double d0 = sqrt(s0 / n), d1 = sqrt(s1 / n);
    const double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
    h[0] = h0;
    h[1] = d1;
    *hf = (float)h0;
  } else {
    const double h0 = h[0], d1 = h[1];
    const double d2 = DIVH ? sqrt(s0 / n) / h0 : sqrt(s0 / n);
    const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 1.0 / order);
    h[2] = fmin(100.0 * h0, h1);
    if (hf) *hf = (float)h[2];  // the first step's coefficient scale, in place for its launches
  }
}

template <class T>
static int initial_step(int64_t n, const T* y0, const T* f0, const T* f1, double atol, double rtol, double order,
                        double* h, float* hf, void* workspace, size_t ws_bytes, void* stream) {
  GNPDE_REQUIRE(n >= 1 && y0 && f0 && h && (f1 || hf) && workspace && order > 0.0, GNPDE_EINVAL,
                "initial_step: bad arguments");
  GNPDE_REQUIRE(ws_bytes >= 2 * sizeof(double) * kDotBlocks, GNPDE_EINVAL, "initial_step: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  const float a = (float)atol, r = (float)rtol;
  const size_t vb = 4 * sizeof(T);
  auto al = [&](const void* p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % vb == 0; };
  const bool v4 = n % 4 == 0 && al(y0) && al(f0) && al(f1);
  if (f1 == nullptr) {
    if (v4)
      init_step_partial_kernel<T, 4, 0><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    else
      init_step_partial_kernel<T, 1, 0><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    GNPDE_LAUNCH_CHECK();
    init_step_final_kernel<0><<<1, kBlock, 0, s>>>(part, kDotBlocks, (double)n, order, h, hf);
  } else {
    if (v4)
      init_step_partial_kernel<T, 4, 1><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    else
      init_step_partial_kernel<T, 1, 1><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    GNPDE_LAUNCH_CHECK();
    init_step_final_kernel<1><<<1, kBlock, 0, s>>>(part, kDotBlocks, (double)n, order, h, hf);
  }
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

// Block partials of the row sums of gnpde_initial_step_rows: part[2b] = sum y (rows_b,
// the y0 channel; rows_a in phase 1), part[2b + 1] = sum rows_a (the f0 channel; 0 in
// phase 1) — the layout init_step_final_kernel reads.
__global__ __launch_bounds__(256) void init_rows_partial_kernel(int64_t n, const double* __restrict__ a,
                                                                 const double* __restrict__ b,
                                                                 double* __restrict__ part) {
  __shared__ double red[kBlock / kWave];
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double sa = 0.0, sb = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += stride) {
    sa += a[i];
    if (b) sb += b[i];
  }
  const double ta = block_sum_f64(sa, red);
  __syncthreads();
  const double tb = b ? block_sum_f64(sb, red) : 0.0;
  if (threadIdx.x == 0) {
    part[2 * blockIdx.x] = b ? tb : ta;
    part[2 * blockIdx.x + 1] = b ? ta : 0.0;
  }
}

template <int VEC, class T>
static int launch_stage_apply(int64_t R, int C, int64_t ld, const T* f, const T* x,
                              const gnpde_stage_epilogue_t& st, hipStream_t s) {
  const int lanes = (int)ceil_div(C, VEC);
  const int64_t waves = [&](int rpw) { return ceil_div(R, (int64_t)rpw); }(lanes <= 16 ? 4 : (lanes <= 32 ? 2 : 1));
  const unsigned grid = (unsigned)std::max<int64_t>(1, ceil_div(waves, kWavesPerBlock));
  const bool light = !st.err_rows && st.n_out <= 1 && st.nk <= 2;
  const bool one_out = !st.err_rows && st.n_out <= 1;  // the dense output over many operands
#define GNPDE_SA(GL)                                                                                  \
  if (light)                                                                                          \
    stage_apply_kernel<VEC, GL, T, 2, 1, false><<<grid, kBlock, 0, s>>>(R, C, ld, f, x, st);          \
  else if (one_out)                                                                                   \
    stage_apply_kernel<VEC, GL, T, GNPDE_STAGE_MAX_K, 1, false><<<grid, kBlock, 0, s>>>(R, C, ld, f, x, st); \
  else                                                                                                \
    stage_apply_kernel<VEC, GL, T, GNPDE_STAGE_MAX_K, 2, true><<<grid, kBlock, 0, s>>>(R, C, ld, f, x, st)
  if (lanes <= 16) {
    GNPDE_SA(16);
  } else if (lanes <= 32) {
    GNPDE_SA(32);
  } else {
    GNPDE_SA(64);
  }
#undef GNPDE_SA
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

template <class T>
static int stage_apply(int64_t R, int64_t C, int64_t ld, const T* f, const T* x, const gnpde_stage_epilogue_t* stage,
                       void* stream) {
  GNPDE_REQUIRE(stage != nullptr && R >= 0 && C >= 1 && ld >= C && C < INT32_MAX, GNPDE_EINVAL,
                "stage_apply: bad arguments");
  int rc = check_stage(*stage);
  if (rc) return rc;
  const gnpde_stage_epilogue_t& st = *stage;
  GNPDE_REQUIRE(!st.dot_rows, GNPDE_EUNSUPPORTED, "stage_apply: dot_rows are fused into the RHS kernels only");
  GNPDE_REQUIRE(!st.dense_out && !st.dense_tab && !st.scale_rows, GNPDE_EUNSUPPORTED,
                "stage_apply: dense_out / dense_tab / scale_rows are fused into the RHS kernel only");
  bool needs_x = st.err_rows && st.err_y1 < 0;
  for (int i = 0; i < st.n_out; ++i)
    GNPDE_REQUIRE(st.o[i].out != reinterpret_cast<const float*>(x), GNPDE_EINVAL, "stage_apply: output %d aliases x",
                  i);
  GNPDE_REQUIRE(!needs_x || x, GNPDE_EINVAL, "stage_apply: the error tolerance reads y1 = x, which is NULL");
  GNPDE_REQUIRE(st.f_lin == 0.f || (x && f), GNPDE_EINVAL, "stage_apply: f_lin needs f and the input x");
  if (R == 0) return GNPDE_OK;
  // widest vector every row array allows
  const int kMax = 16 / (int)sizeof(T);
  int vec = 1;
  for (int v = kMax; v > 1; v >>= 1) {
    const size_t bytes = (size_t)v * sizeof(T);
    auto al = [&](const void* p) { return p == nullptr || (reinterpret_cast<uintptr_t>(p) % bytes) == 0; };
    bool ok = C % v == 0 && ld % v == 0 && al(f) && al(x) && al(st.f_out) && al(st.err.base) && al(st.err_y0);
    for (int i = 0; i < st.n_out; ++i) ok = ok && al(st.o[i].out) && al(st.o[i].base);
    for (int j = 0; j < st.nk; ++j) ok = ok && al(st.k[j]);
    if (ok) {
      vec = v;
      break;
    }
  }
  hipStream_t s = as_stream(stream);
  const int c = (int)C;
  switch (vec) {
    case 8:
      if constexpr (sizeof(T) == 2) return launch_stage_apply<8, T>(R, c, ld, f, x, st, s);
      [[fallthrough]];
    case 4: return launch_stage_apply<4, T>(R, c, ld, f, x, st, s);
    case 2: return launch_stage_apply<2, T>(R, c, ld, f, x, st, s);
    default: return launch_stage_apply<1, T>(R, c, ld, f, x, st, s);
  }
}

}  // namespace gnpde

using namespace gnpde;

extern "C" int gnpde_stage_apply_f32(int64_t R, int64_t C, int64_t ld, const float* f, const float* x,
                                     const gnpde_stage_epilogue_t* stage, void* stream) {
  return stage_apply<float>(R, C, ld, f, x, stage, stream);
}

extern "C" int gnpde_stage_apply_bf16(int64_t R, int64_t C, int64_t ld, const uint16_t* f, const uint16_t* x,
                                      const gnpde_stage_epilogue_t* stage, void* stream) {
  return stage_apply<bf16>(R, C, ld, reinterpret_cast<const bf16*>(f), reinterpret_cast<const bf16*>(x), stage,
                           stream);
}

extern "C" int gnpde_rows_copy(const void* src, int64_t rows, int64_t row_bytes, const int64_t* order, void* dst,
                               void* dst_copy, void* stream) {
  GNPDE_REQUIRE(rows >= 0 && row_bytes >= 0 && src && dst, GNPDE_EINVAL, "rows_copy: bad arguments");
  GNPDE_REQUIRE(row_bytes % 16 == 0 && aligned16(src) && aligned16(dst) && (!dst_copy || aligned16(dst_copy)),
                GNPDE_EUNSUPPORTED, "rows_copy: rows of %lld bytes / pointers not 16-byte aligned",
                (long long)row_bytes);
  GNPDE_REQUIRE(src != dst && src != dst_copy, GNPDE_EINVAL, "rows_copy: src aliases an output");
  const int64_t v4 = row_bytes / 16;
  if (rows == 0 || v4 == 0) return GNPDE_OK;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(rows * v4, kBlock), 16384));
  hipStream_t s = as_stream(stream);
  const uint4* sp = reinterpret_cast<const uint4*>(src);
  uint4* dp = reinterpret_cast<uint4*>(dst);
  uint4* cp = reinterpret_cast<uint4*>(dst_copy);
  if (order && cp)
    rows_copy_kernel<true, true><<<grid, kBlock, 0, s>>>(sp, rows, v4, order, dp, cp);
  else if (order)
    rows_copy_kernel<true, false><<<grid, kBlock, 0, s>>>(sp, rows, v4, order, dp, cp);
  else if (cp)
    rows_copy_kernel<false, true><<<grid, kBlock, 0, s>>>(sp, rows, v4, order, dp, cp);
  else
    rows_copy_kernel<false, false><<<grid, kBlock, 0, s>>>(sp, rows, v4, order, dp, cp);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" size_t gnpde_dot_workspace_bytes(void) { return sizeof(double) * kDotBlocks; }

extern "C" int gnpde_sum_f64(int64_t n, const double* v, double* out, int accumulate, void* workspace,
                             size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(n >= 0 && (v || n == 0) && out && workspace, GNPDE_EINVAL, "sum_f64: NULL pointer or bad n");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_dot_workspace_bytes(), GNPDE_EINVAL, "sum_f64: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  sum_partial_kernel<<<kDotBlocks, kBlock, 0, s>>>(n, v, part);
  GNPDE_LAUNCH_CHECK();
  sum_final_kernel<<<1, kBlock, 0, s>>>(part, kDotBlocks, out, accumulate);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" int gnpde_dot_f64(int64_t n, const float* a, const float* b, double* out, void* workspace,
                             size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(n >= 0 && a && b && out && workspace, GNPDE_EINVAL, "dot: NULL pointer or bad n");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_dot_workspace_bytes(), GNPDE_EINVAL, "dot: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  const bool vec4 = n % 4 == 0 && aligned16(a) && aligned16(b);
  if (vec4)
    dot_partial_kernel<true><<<kDotBlocks, kBlock, 0, s>>>(n, a, b, part);
  else
    dot_partial_kernel<false><<<kDotBlocks, kBlock, 0, s>>>(n, a, b, part);
  GNPDE_LAUNCH_CHECK();
  dot_final_kernel<<<1, kBlock, 0, s>>>(part, kDotBlocks, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" int gnpde_rk_combine_f32(int64_t n, const float* y0, int nk, const float* const* ks, const double* coef,
                                    double scale, float* out, void* stream) {
  GNPDE_REQUIRE(n >= 0 && out, GNPDE_EINVAL, "rk_combine: bad args");
  GNPDE_REQUIRE(nk >= 0 && nk <= kMaxStages, GNPDE_EUNSUPPORTED, "rk_combine: nk=%d > %d", nk, kMaxStages);
  GNPDE_REQUIRE(nk == 0 || (ks && coef), GNPDE_EINVAL, "rk_combine: NULL ks/coef");
  if (n == 0) return GNPDE_OK;
  CombineArgs a;
  a.nk = nk;
  bool vec4 = (n % 4 == 0) && (y0 == nullptr || aligned16(y0)) && aligned16(out);
  for (int j = 0; j < kMaxStages; ++j) {
    a.k[j] = j < nk ? ks[j] : nullptr;
    a.c[j] = j < nk ? (float)(scale * coef[j]) : 0.f;
    if (j < nk) {
      GNPDE_REQUIRE(ks[j] != nullptr, GNPDE_EINVAL, "rk_combine: ks[%d] is NULL", j);
      vec4 = vec4 && aligned16(ks[j]);
    }
  }
  const int64_t work = vec4 ? n / 4 : n;
  const unsigned grid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(ceil_div(work, kBlock), 8192));
  hipStream_t s = as_stream(stream);
  if (vec4)
    rk_combine_kernel<true><<<grid, kBlock, 0, s>>>(n, y0, a, out);
  else
    rk_combine_kernel<false><<<grid, kBlock, 0, s>>>(n, y0, a, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" size_t gnpde_initial_step_workspace_bytes(void) { return 2 * sizeof(double) * kDotBlocks; }

extern "C" int gnpde_initial_step_f32(int64_t n, const float* y0, const float* f0, const float* f1, double atol,
                                      double rtol, double order, double* h, float* hf, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  return initial_step<float>(n, y0, f0, f1, atol, rtol, order, h, hf, workspace, workspace_bytes, stream);
}

// phase 1 of the initial step from v = L f0 (the linear part of an affine RHS on f0):
// d2 = rms(v / scale), the quotient in fp32 as gnpde_initial_step_f32's
template <class T>
static int initial_step_lin(int64_t n, const T* y0, const T* v, double atol, double rtol, double order, double* h,
                            float* hf, void* workspace, size_t ws_bytes, void* stream) {
  GNPDE_REQUIRE(n >= 1 && y0 && v && h && workspace && order > 0.0, GNPDE_EINVAL, "initial_step_lin: bad arguments");
  GNPDE_REQUIRE(ws_bytes >= 2 * sizeof(double) * kDotBlocks, GNPDE_EINVAL, "initial_step_lin: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  const float a = (float)atol, r = (float)rtol;
  const size_t vb = 4 * sizeof(T);
  const bool v4 = n % 4 == 0 && reinterpret_cast<uintptr_t>(y0) % vb == 0 && reinterpret_cast<uintptr_t>(v) % vb == 0;
  if (v4)
    init_step_partial_kernel<T, 4, 2><<<kDotBlocks, kBlock, 0, s>>>(n, y0, nullptr, v, a, r, part);
  else
    init_step_partial_kernel<T, 1, 2><<<kDotBlocks, kBlock, 0, s>>>(n, y0, nullptr, v, a, r, part);
  GNPDE_LAUNCH_CHECK();
  init_step_final_kernel<1, false><<<1, kBlock, 0, s>>>(part, kDotBlocks, (double)n, order, h, hf);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" int gnpde_initial_step_lin_f32(int64_t n, const float* y0, const float* v, double atol, double rtol,
                                          double order, double* h, float* hf, void* workspace, size_t workspace_bytes,
                                          void* stream) {
  return initial_step_lin<float>(n, y0, v, atol, rtol, order, h, hf, workspace, workspace_bytes, stream);
}

extern "C" int gnpde_initial_step_lin_bf16(int64_t n, const uint16_t* y0, const uint16_t* v, double atol, double rtol,
                                           double order, double* h, float* hf, void* workspace,
                                           size_t workspace_bytes, void* stream) {
  return initial_step_lin<bf16>(n, reinterpret_cast<const bf16*>(y0), reinterpret_cast<const bf16*>(v), atol, rtol,
                                order, h, hf, workspace, workspace_bytes, stream);
}

extern "C" int gnpde_initial_step_rows(int64_t nrows, const double* rows_a, const double* rows_b, double n,
                                       double order, double* h, float* hf, void* workspace, size_t workspace_bytes,
                                       void* stream) {
  GNPDE_REQUIRE(nrows >= 1 && rows_a && h && n > 0.0 && order > 0.0 && workspace,
                GNPDE_EINVAL, "initial_step_rows: bad arguments");
  GNPDE_REQUIRE(rows_b == nullptr || hf != nullptr, GNPDE_EINVAL, "initial_step_rows: phase 0 needs hf");
  GNPDE_REQUIRE(workspace_bytes >= 2 * sizeof(double) * kDotBlocks, GNPDE_EINVAL,
                "initial_step_rows: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  init_rows_partial_kernel<<<kDotBlocks, kBlock, 0, s>>>(nrows, rows_a, rows_b, part);
  GNPDE_LAUNCH_CHECK();
  if (rows_b)
    init_step_final_kernel<0><<<1, kBlock, 0, s>>>(part, kDotBlocks, n, order, h, hf);
  else
    init_step_final_kernel<1, false><<<1, kBlock, 0, s>>>(part, kDotBlocks, n, order, h, hf);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

extern "C" int gnpde_initial_step_bf16(int64_t n, const uint16_t* y0, const uint16_t* f0, const uint16_t* f1,
                                       double atol, double rtol, double order, double* h, float* hf, void* workspace,
                                       size_t workspace_bytes, void* stream) {
  return initial_step<bf16>(n, reinterpret_cast<const bf16*>(y0), reinterpret_cast<const bf16*>(f0),
                            reinterpret_cast<const bf16*>(f1), atol, rtol, order, h, hf, workspace, workspace_bytes,
                            stream);
}

// The two squared sums of init_step_partial_kernel, stored as they are (the mixed norm
// of the adjoint's augmented state combines them per component on the host)
__global__ __launch_bounds__(256) void pair_sum_final_kernel(const double* __restrict__ part, int nb,
                                                              double* __restrict__ out) {
  __shared__ double red[kBlock / kWave];
  double a0 = 0.0, a1 = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) {
    a0 += part[2 * i];
    a1 += part[2 * i + 1];
  }
  const double s0 = block_sum_f64(a0, red);
  __syncthreads();
  const double s1 = block_sum_f64(a1, red);
  if (threadIdx.x == 0) {
    out[0] = s0;
    out[1] = s1;
  }
}

extern "C" int gnpde_scaled_sq_sums_f32(int64_t n, const float* y0, const float* f0, const float* f1, double atol,
                                        double rtol, double* out, void* workspace, size_t ws_bytes, void* stream) {
  GNPDE_REQUIRE(n >= 1 && y0 && f0 && out && workspace, GNPDE_EINVAL, "scaled_sq_sums: bad arguments");
  GNPDE_REQUIRE(ws_bytes >= 2 * sizeof(double) * kDotBlocks, GNPDE_EINVAL, "scaled_sq_sums: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  const float a = (float)atol, r = (float)rtol;
  auto al = [&](const void* p) { return p == nullptr || reinterpret_cast<uintptr_t>(p) % 16 == 0; };
  const bool v4 = n % 4 == 0 && al(y0) && al(f0) && al(f1);
  if (f1 == nullptr) {
    if (v4)
      init_step_partial_kernel<float, 4, 0><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    else
      init_step_partial_kernel<float, 1, 0><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
  } else {
    if (v4)
      init_step_partial_kernel<float, 4, 1><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
    else
      init_step_partial_kernel<float, 1, 1><<<kDotBlocks, kBlock, 0, s>>>(n, y0, f0, f1, a, r, part);
  }
  GNPDE_LAUNCH_CHECK();
  pair_sum_final_kernel<<<1, kBlock, 0, s>>>(part, kDotBlocks, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

// Segment sums: kSegSumBlocks blocks per segment (blockIdx.y = segment), each thread
// summing a fixed stride of its segment in order, a fixed tree per block, then one
// block per segment summing its block partials in order (deterministic).
constexpr int kSegSumBlocks = 128;

__global__ __launch_bounds__(256) void seg_sum_partial_kernel(int64_t len, const double* __restrict__ v,
                                                               double* __restrict__ part) {
  __shared__ double red[kBlock / kWave];
  const double* seg = v + (int64_t)blockIdx.y * len;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  double acc = 0.0;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < len; i += stride) acc += seg[i];
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) part[(int64_t)blockIdx.y * gridDim.x + blockIdx.x] = t;
}

__global__ __launch_bounds__(256) void seg_sum_final_kernel(const double* __restrict__ part, int nb,
                                                             double* __restrict__ out) {
  __shared__ double red[kBlock / kWave];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[(int64_t)blockIdx.x * nb + i];
  const double t = block_sum_f64(acc, red);
  if (threadIdx.x == 0) out[blockIdx.x] = t;
}

extern "C" size_t gnpde_segment_sums_workspace_bytes(int64_t nseg) {
  return sizeof(double) * (size_t)kSegSumBlocks * (size_t)(nseg > 0 ? nseg : 0);
}

extern "C" int gnpde_segment_sums_f64(int64_t nseg, int64_t len, const double* v, double* out, void* workspace,
                                      size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(nseg >= 0 && nseg <= 65535 && len >= 0 && out && workspace && (v || nseg * len == 0), GNPDE_EINVAL,
                "segment_sums: bad arguments");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_segment_sums_workspace_bytes(nseg), GNPDE_EINVAL,
                "segment_sums: workspace too small");
  if (nseg == 0) return GNPDE_OK;
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  seg_sum_partial_kernel<<<dim3(kSegSumBlocks, (unsigned)nseg), kBlock, 0, s>>>(len, v, part);
  GNPDE_LAUNCH_CHECK();
  seg_sum_final_kernel<<<(unsigned)nseg, kBlock, 0, s>>>(part, kSegSumBlocks, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

// torchdiffeq's step-size controller (rk_common.py _optimal_step_size, the adaptive
// loop's accept test) on the device, fused with the last level of the step's error
// reduction (the same fixed order as gnpde_sum_f64): the host reads rec = {error
// ratio, dt of the step, dt of the next step, squared error sum} once, and the next
// step's coefficient scale is already in place (no host fill between two replayed
// steps, no separate sum launch).
__global__ __launch_bounds__(256) void adaptive_control_kernel(const double* __restrict__ part, int nb, double n,
                                                                double order, double safety, double ifactor,
                                                                double dfactor, double* dt, float* scale, double* rec,
                                                                double* t) {
  __shared__ double red[kBlock / kWave];
  double acc = 0.0;
  for (int i = threadIdx.x; i < nb; i += blockDim.x) acc += part[i];
  const double e2 = block_sum_f64(acc, red);
  if (threadIdx.x != 0) return;
  const double h = *dt;
  const double ratio = n > 0.0 ? sqrt(e2 / n) : 0.0;
  double next;
  if (ratio == 0.0) {
    next = h * ifactor;
  } else {
    const double df = ratio < 1.0 ? 1.0 : dfactor;
    next = h * fmin(ifactor, fmax(safety / pow(ratio, 1.0 / order), df));
  }
  rec[0] = ratio;
  rec[1] = h;
  rec[2] = next;
  rec[3] = e2;
  *dt = next;
  *scale = (float)next;
  if (t && ratio <= 1.0) *t += h;  // the accepted step's end: the next step's start (dense_t)
}

extern "C" int gnpde_adaptive_control(int64_t nrows, const double* err_rows, double n, double order, double safety,
                                      double ifactor, double dfactor, double* dt, float* scale, double* rec,
                                      double* t, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(nrows >= 0 && (err_rows || nrows == 0) && dt && scale && rec && workspace && order > 0.0,
                GNPDE_EINVAL, "adaptive_control: bad arguments");
  GNPDE_REQUIRE(workspace_bytes >= sizeof(double) * kDotBlocks, GNPDE_EINVAL, "adaptive_control: workspace too small");
  hipStream_t s = as_stream(stream);
  double* part = static_cast<double*>(workspace);
  sum_partial_kernel<<<kDotBlocks, kBlock, 0, s>>>(nrows, err_rows, part);
  GNPDE_LAUNCH_CHECK();
  adaptive_control_kernel<<<1, kBlock, 0, s>>>(part, kDotBlocks, n, order, safety, ifactor, dfactor, dt, scale, rec,
                                               t);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}
