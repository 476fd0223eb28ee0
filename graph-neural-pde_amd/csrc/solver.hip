// solver.hip — fused Runge-Kutta stage combination: one streaming pass for
// y0 + dt * sum_j b_j k_j (torchdiffeq's rk4_alt_step_func / _runge_kutta_step
// do it with several elementwise torch kernels per stage).
#include "common.hpp"

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

}  // namespace gnpde

using namespace gnpde;

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
