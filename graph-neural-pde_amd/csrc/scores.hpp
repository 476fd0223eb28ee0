// scores.hpp — attention edge scores (function_transformer_attention.py:246-259).
#pragma once
#include "common.hpp"

namespace gnpde {

// Scores of one (src, dst) pair for one head (function_transformer_attention.py:246-259).
__device__ __forceinline__ float pair_score(int mode, const float* __restrict__ qi, const float* __restrict__ kj,
                                            int dk, float p0, float p1) {
  if (mode == GNPDE_SCORE_DOT) {
    float s = 0.f;
    for (int d = 0; d < dk; ++d) s = fmaf(qi[d], kj[d], s);
    return s * rsqrtf((float)dk) ;
  } else if (mode == GNPDE_SCORE_EXP_KERNEL) {
    float s = 0.f;
    for (int d = 0; d < dk; ++d) {
      const float t = qi[d] - kj[d];
      s = fmaf(t, t, s);
    }
    return p0 * p0 * expf(-(s / (2.0f * p1 * p1)));
  } else {  // cosine / pearson: torch>=1.12 CosineSimilarity, each operand / max(norm, eps)
    float mq = 0.f, mk = 0.f;
    if (mode == GNPDE_SCORE_PEARSON) {
      for (int d = 0; d < dk; ++d) { mq += qi[d]; mk += kj[d]; }
      mq /= (float)dk;
      mk /= (float)dk;
    }
    float nq = 0.f, nk = 0.f, dot = 0.f;
    for (int d = 0; d < dk; ++d) {
      const float a = qi[d] - mq, b = kj[d] - mk;
      nq = fmaf(a, a, nq);
      nk = fmaf(b, b, nk);
      dot = fmaf(a, b, dot);
    }
    const float den = fmaxf(sqrtf(nq), 1e-5f) * fmaxf(sqrtf(nk), 1e-5f);
    return dot / den;
  }
}

struct ScoreArgs {
  int mode;
  int H;
  int dk;
  const double* __restrict__ cs;  // [R,H] reference-mode node scores (fp64)
  const float* __restrict__ q;    // [R,ldqk] per-edge modes
  const float* __restrict__ k;
  int64_t ldqk;
  float p0, p1;

  // score of edge src->dst, head h, as double (exact for the fp32 modes)
  __device__ __forceinline__ double score(int src, int dst, int h) const {
    if (mode == GNPDE_SCORE_REFERENCE) return cs[(int64_t)src * H + h];
    if (mode == GNPDE_SCORE_UNIFORM) return 0.0;
    return (double)pair_score(mode, q + (int64_t)src * ldqk + h * dk, k + (int64_t)dst * ldqk + h * dk, dk, p0, p1);
  }
};

}  // namespace gnpde
