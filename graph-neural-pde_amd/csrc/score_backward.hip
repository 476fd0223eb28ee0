// score_backward.hip — backward of the per-edge attention scores
// (src/function_transformer_attention.py:246-259) for the score types whose
// derivative is not a plain product: exp_kernel, cosine_sim, pearson (and the
// per-edge scaled_dot, through the same kernel).
//
// Given g_s[e,h] = dL/ds (the edge-softmax backward's output, COO [E,H]), the
// gradient reaching the projection of node r is, per head h and element d,
//
//   g[r, h*dk + d] = own'_d * sum_e g_s a_own(e)  +  sum_e g_s a_oth(e) * oth'_d(e)
//
// over the edges e of r's group (source-grouped CSR for the q side, the CSC for
// the k side), because every score derivative is a combination of the two
// operands (own = the row's q or k, oth = the other endpoint's k or q; ' =
// centred for pearson, whose centring projects the gradient back onto
// zero-mean vectors that are already zero-mean):
//
//   scaled_dot  s = q.k / sqrt(dk)                 a_own = 0,        a_oth = 1/sqrt(dk)
//   exp_kernel  s = ov^2 exp(-|q-k|^2 / (2 ls^2))   a_own = -s/ls^2,  a_oth = s/ls^2
//   cosine      s = q.k / (max(|q|,eps) max(|k|,eps))  a_own = -s/|own|^2, a_oth = 1/(|q| |k|)
//   pearson     cosine of the centred operands
//
// exp_kernel's parameters also get per-edge terms (COO order, summed by the
// caller in fp64): ds/dov = 2 s / ov, ds/dls = s |q-k|^2 / ls^3.
//
// One wavefront per row (64-thread workgroups); lane j holds elements j, j+64, ...
// of the att-wide rows; per-head sums meet in LDS (any dk).  Fixed summation
// order everywhere: deterministic.
#include "common.hpp"

namespace gnpde {

namespace {

constexpr int kMaxAtt = 1024;
constexpr int kPass = kMaxAtt / kWave;  // elements per lane
constexpr float kCosEps = 1e-5f;        // torch.nn.CosineSimilarity(eps=1e-5), :251, :258

struct ScoreGradArgs {
  const int* rowptr;
  const int* col;
  const int* perm;
  int64_t R;
  int side;  // 0: rows are sources, own = q; 1: rows are destinations, own = k
  int mode;
  int H, dk, att;
  const float* q;
  const float* k;
  int64_t ldqk;
  float p0, p1;
  const float* gs;  // [E, H] COO
  float* out;       // [R, ldo]
  int64_t ldo;
  float* gp;  // [E, 2H] COO or NULL
};

// per-head sum of v over the dk elements of each head, via the wave's LDS row
__device__ __forceinline__ void head_sums(float* lds, const float (&v)[kPass], int att, int dk, float (&out)[kPass]) {
  const int lane = threadIdx.x;
#pragma unroll
  for (int t = 0; t < kPass; ++t) {
    const int j = lane + t * kWave;
    if (j < att) lds[j] = v[t];
  }
  __syncthreads();
#pragma unroll
  for (int t = 0; t < kPass; ++t) {
    const int j = lane + t * kWave;
    float s = 0.f;
    if (j < att) {
      const int h0 = (j / dk) * dk;
      for (int d = 0; d < dk; ++d) s += lds[h0 + d];
    }
    out[t] = s;
  }
  __syncthreads();
}

__global__ __launch_bounds__(64) void score_grad_kernel(ScoreGradArgs a) {
  __shared__ float lds[kMaxAtt];
  const int lane = threadIdx.x;
  const int npass = (a.att + kWave - 1) / kWave;
  const float* own_base = a.side == 0 ? a.q : a.k;
  const float* oth_base = a.side == 0 ? a.k : a.q;
  const float rdk = 1.0f / (float)a.dk;
  for (int64_t r = blockIdx.x; r < a.R; r += gridDim.x) {
    float own[kPass], acc[kPass], A[kPass];
#pragma unroll
    for (int t = 0; t < kPass; ++t) {
      const int j = lane + t * kWave;
      own[t] = (t < npass && j < a.att) ? own_base[r * a.ldqk + j] : 0.f;
      acc[t] = 0.f;
      A[t] = 0.f;
    }
    if (a.mode == GNPDE_SCORE_PEARSON) {
      float m[kPass];
      head_sums(lds, own, a.att, a.dk, m);
#pragma unroll
      for (int t = 0; t < kPass; ++t) own[t] -= m[t] * rdk;
    }
    float own_n[kPass];
    {
      float sq[kPass];
#pragma unroll
      for (int t = 0; t < kPass; ++t) sq[t] = own[t] * own[t];
      head_sums(lds, sq, a.att, a.dk, own_n);
    }
    const int b = a.rowptr[r], e_end = a.rowptr[r + 1];
    for (int p = b; p < e_end; ++p) {
      const int oth_node = a.col[p];
      const int64_t e = a.perm[p];
      float oth[kPass];
#pragma unroll
      for (int t = 0; t < kPass; ++t) {
        const int j = lane + t * kWave;
        oth[t] = (t < npass && j < a.att) ? oth_base[(int64_t)oth_node * a.ldqk + j] : 0.f;
      }
      if (a.mode == GNPDE_SCORE_PEARSON) {
        float m[kPass];
        head_sums(lds, oth, a.att, a.dk, m);
#pragma unroll
        for (int t = 0; t < kPass; ++t) oth[t] -= m[t] * rdk;
      }
      float prod[kPass], S1[kPass], S2[kPass];
      // S1: q.k (dot / cosine / pearson) or |q - k|^2 (exp_kernel); S2: |oth|^2
#pragma unroll
      for (int t = 0; t < kPass; ++t) {
        const float d = own[t] - oth[t];
        prod[t] = a.mode == GNPDE_SCORE_EXP_KERNEL ? d * d : own[t] * oth[t];
      }
      head_sums(lds, prod, a.att, a.dk, S1);
      const bool cos = a.mode == GNPDE_SCORE_COSINE || a.mode == GNPDE_SCORE_PEARSON;
      if (cos) {
#pragma unroll
        for (int t = 0; t < kPass; ++t) prod[t] = oth[t] * oth[t];
        head_sums(lds, prod, a.att, a.dk, S2);
      }
#pragma unroll
      for (int t = 0; t < kPass; ++t) {
        const int j = lane + t * kWave;
        if (t >= npass || j >= a.att) continue;
        const int h = j / a.dk;
        const float g = a.gs[e * a.H + h];
        float a_own, a_oth;
        if (a.mode == GNPDE_SCORE_DOT) {
          a_own = 0.f;
          a_oth = rsqrtf((float)a.dk);
        } else if (a.mode == GNPDE_SCORE_EXP_KERNEL) {
          const float s = a.p0 * a.p0 * expf(-(S1[t] / (2.0f * a.p1 * a.p1)));
          a_own = -s / (a.p1 * a.p1);
          a_oth = -a_own;
          if (a.gp != nullptr && j % a.dk == 0) {  // one lane per head: the parameter terms
            a.gp[e * 2 * a.H + h] = g * 2.0f * s / a.p0;
            a.gp[e * 2 * a.H + a.H + h] = g * s * S1[t] / (a.p1 * a.p1 * a.p1);
          }
        } else {
          const float no = fmaxf(sqrtf(own_n[t]), kCosEps), nt = fmaxf(sqrtf(S2[t]), kCosEps);
          const float s = S1[t] / (no * nt);
          a_own = -s / (no * no);
          a_oth = 1.0f / (no * nt);
        }
        A[t] = fmaf(g, a_own, A[t]);
        acc[t] = fmaf(g * a_oth, oth[t], acc[t]);
      }
    }
#pragma unroll
    for (int t = 0; t < kPass; ++t) {
      const int j = lane + t * kWave;
      if (t < npass && j < a.att) a.out[r * a.ldo + j] = fmaf(own[t], A[t], acc[t]);
    }
  }
}

}  // namespace
}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_score_grad_f32(const int32_t* rowptr, const int32_t* col, const int32_t* perm, int64_t R, int64_t nnz,
                         int side, int mode, int64_t heads, int64_t dk, const float* q, const float* k, int64_t ldqk,
                         float score_p0, float score_p1, const float* gs, float* out, int64_t ldo, float* gp,
                         void* stream) {
  GNPDE_REQUIRE(side == 0 || side == 1, GNPDE_EINVAL, "score_grad: side must be 0 or 1");
  GNPDE_REQUIRE(mode == GNPDE_SCORE_DOT || mode == GNPDE_SCORE_EXP_KERNEL || mode == GNPDE_SCORE_COSINE ||
                    mode == GNPDE_SCORE_PEARSON,
                GNPDE_EUNSUPPORTED, "score_grad: per-edge score modes only (got %d)", mode);
  GNPDE_REQUIRE(heads >= 1 && dk >= 1 && heads * dk <= kMaxAtt, GNPDE_EUNSUPPORTED,
                "score_grad: attention_dim %lld > %d", (long long)(heads * dk), kMaxAtt);
  GNPDE_REQUIRE(R >= 1 && nnz >= 0 && ldqk >= heads * dk && ldo >= heads * dk, GNPDE_EINVAL, "score_grad: bad sizes");
  GNPDE_REQUIRE(rowptr && out && (nnz == 0 || (col && perm && q && k && gs)), GNPDE_EINVAL,
                "score_grad: NULL pointer");
  GNPDE_REQUIRE(R < (int64_t)INT32_MAX && nnz < (int64_t)INT32_MAX, GNPDE_EUNSUPPORTED, "score_grad: too large");
  ScoreGradArgs a{rowptr, col, perm, R, side, mode, (int)heads, (int)dk, (int)(heads * dk), q, k, ldqk,
                  score_p0, score_p1, gs, out, ldo, gp};
  const int64_t grid = R < 65536 ? R : 65536;
  score_grad_kernel<<<(unsigned)grid, kWave, 0, as_stream(stream)>>>(a);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
