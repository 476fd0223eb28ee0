// rhs.hip — the C ABI of K1 (aggregate.hpp): the Laplacian SpMM RHS in fp32 and
// bf16 storage, and the fused-weight attention RHS (gnpde_attn_ref_rhs_f32).
// The score / softmax pieces around it are in node_scores.hip.
#include "aggregate.hpp"
#include "rhs_host.hpp"

namespace gnpde {

int bf16_vec_cap() {
  if constexpr (!GNPDE_EXPERIMENTS) return 4;
  static const int v = [] {
    // cap of the elements per lane (default 4 = 8-byte gathers); rows of 129-256 columns take
    // 16-byte gathers anyway (epi_vec_width) so that they fit the two-rows-per-wavefront geometry
    const char* e = std::getenv("GNPDE_BF16_VEC");
    const int c = e ? std::atoi(e) : 4;
    return (c == 1 || c == 2 || c == 8) ? c : 4;
  }();
  return v;
}

bool hub_inlaunch() {
  if constexpr (!GNPDE_EXPERIMENTS) return true;
  static const bool v = [] {
    const char* e = std::getenv("GNPDE_HUB_FIXUP");
    return !(e && std::atoi(e) == 1);
  }();
  return v;
}

int agg_variant() {
  if constexpr (!GNPDE_EXPERIMENTS) return 0;
  static const int v = [] {
    const char* e = std::getenv("GNPDE_AGG_VARIANT");
    return e ? std::atoi(e) : 0;
  }();
  return v;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_spmm_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                       const int32_t* col, const float* w, int64_t C, const float* x, int64_t ldx, const float* x0,
                       int64_t ldx0, const float* alpha, const float* beta, int flags, float* f, int64_t ldf,
                       float* partials, int64_t n_slots, const gnpde_stage_epilogue_t* stage, void* stream) {
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf, stage);
  int rc = check_epi(ep, C, n_heavy, partials, n_slots);
  if (rc) return rc;
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0, GNPDE_EINVAL, "spmm_rhs: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && w), GNPDE_EINVAL, "spmm_rhs: NULL plan/col/w");
  PlainWeights wp{w};
  return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
}

int gnpde_spmm_rhs_bf16(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                        const int32_t* col, const float* w, int64_t C, const uint16_t* x, int64_t ldx,
                        const uint16_t* x0, int64_t ldx0, const float* alpha, const float* beta, int flags, uint16_t* f,
                        int64_t ldf, float* partials, int64_t n_slots, const gnpde_stage_epilogue_t* stage,
                        void* stream) {
  GNPDE_REQUIRE(!stage || !stage->dot_rows, GNPDE_EUNSUPPORTED, "spmm_rhs_bf16: stage dot terms are fp32 only");
  const Epi ep = make_epi(reinterpret_cast<const float*>(x), ldx, reinterpret_cast<const float*>(x0), ldx0, alpha,
                          beta, flags, reinterpret_cast<float*>(f), ldf, stage);
  int rc = check_epi(ep, C, n_heavy, partials, n_slots);
  if (rc) return rc;
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0, GNPDE_EINVAL, "spmm_rhs_bf16: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && w), GNPDE_EINVAL, "spmm_rhs_bf16: NULL plan/col/w");
  PlainWeights wp{w};
  return launch_agg<PlainWeights, bf16>(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
}

int gnpde_attn_ref_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                           const int32_t* col, const double* cs, const double* m, const float* rl, const float* mr,
                           int64_t heads,
                           int64_t C, const float* x, int64_t ldx, const float* x0, int64_t ldx0, const float* alpha,
                           const float* beta, int flags, float* f, int64_t ldf, float* partials, int64_t n_slots,
                           const gnpde_stage_epilogue_t* stage, void* stream) {
  const Epi ep = make_epi(x, ldx, x0, ldx0, alpha, beta, flags, f, ldf, stage);
  int rc = check_epi(ep, C, n_heavy, partials, n_slots);
  if (rc) return rc;
  GNPDE_REQUIRE(heads >= 1 && heads <= 16, GNPDE_EUNSUPPORTED, "attn_ref_rhs: heads=%lld not in [1,16]",
                (long long)heads);
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && n_heavy >= 0, GNPDE_EINVAL, "attn_ref_rhs: bad item counts");
  GNPDE_REQUIRE(n_items == 0 || (items && col && cs && ((m && rl) || mr)), GNPDE_EINVAL,
                "attn_ref_rhs: NULL plan/col/cs/statistics");
  if (mr) {
    GNPDE_REQUIRE(heads == 2 && aligned16(mr), GNPDE_EUNSUPPORTED,
                  "attn_ref_rhs: packed statistics records are read for two heads, 16-byte aligned");
    RefDstSoftmaxWeights<2, true, true> wp{cs, nullptr, nullptr, 2, mr};
    return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
  }
  if (heads <= 2) {  // separate m / rl arrays (the packed records above are the fast path)
    RefDstSoftmaxWeights<2> wp{cs, m, rl, (int)heads, nullptr};
    return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
  }
  RefDstSoftmaxWeights<0> wp{cs, m, rl, (int)heads, nullptr};
  return launch_agg(items, n_items, heavy, n_heavy, col, wp, C, ep, partials, as_stream(stream));
}

}  // extern "C"
