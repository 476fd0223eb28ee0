// scores.hpp — attention edge scores (function_transformer_attention.py:246-259).
//
// Two evaluation shapes:
//  * lane mode: one lane evaluates a whole (src, dst) pair for one head
//    (reference / uniform modes: a node-score gather; fallback for odd dk);
//  * team mode: T lanes cooperate on one edge, lane t holding VEC consecutive
//    elements of the att-wide q/k rows (coalesced 16-byte gathers); the S =
//    dk/VEC lanes of a head reduce with xor shuffles, so every lane ends with
//    its own head's score.
#pragma once
#include "common.hpp"

namespace gnpde {

__device__ __forceinline__ float pair_score(int mode, const float* __restrict__ qi, const float* __restrict__ kj,
                                            int dk, float p0, float p1) {
  if (mode == GNPDE_SCORE_DOT) {
    float s = 0.f;
    for (int d = 0; d < dk; ++d) s = fmaf(qi[d], kj[d], s);
    return s * rsqrtf((float)dk);
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
      for (int d = 0; d < dk; ++d) {
        mq += qi[d];
        mk += kj[d];
      }
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

// ------------------------------------------------------------------ online softmax state
// (max, sum-exp) pushed one score at a time and merged pairwise in a fixed
// order (deterministic).  fp64 max for the reference mode's fp64 node scores;
// the float twin serves the fp32 per-edge scores of the fused kernel.
// Branch-free (selects, one exp): the same values as the two-branch form, and no
// basic blocks between a wave's gathers and their uses — behind branches the
// compiler issued each score load just before its push (the 8-head long items of
// the Cora-sized CSC statistics waited out one load latency per push).
#ifndef GNPDE_PUSH_SELECT
#define GNPDE_PUSH_SELECT 1
#endif
__device__ __forceinline__ void online_push(double& M, float& L, double s) {
  if constexpr (GNPDE_PUSH_SELECT) {
    const bool gt = s > M;
    const float e = expf((float)(gt ? M - s : s - M));
    const float up = (M == -INFINITY ? 0.f : L * e) + 1.f;
    L = gt ? up : L + e;
    M = gt ? s : M;
    return;
  }
  if (s > M) {
    L = (M == -INFINITY ? 0.f : L * expf((float)(M - s))) + 1.f;
    M = s;
  } else {
    L += expf((float)(s - M));
  }
}

__device__ __forceinline__ void online_merge(double& M, float& L, double M2, float L2) {
  const double Mn = fmax(M, M2);
  if (Mn == -INFINITY) return;
  const float a = (M == -INFINITY) ? 0.f : L * expf((float)(M - Mn));
  const float b = (M2 == -INFINITY) ? 0.f : L2 * expf((float)(M2 - Mn));
  L = a + b;
  M = Mn;
}

__device__ __forceinline__ void online_push(float& M, float& L, float s) {
  if (s > M) {
    L = (M == -INFINITY ? 0.f : L * expf(M - s)) + 1.f;
    M = s;
  } else {
    L += expf(s - M);
  }
}

__device__ __forceinline__ void online_merge(float& M, float& L, float M2, float L2) {
  const float Mn = fmaxf(M, M2);
  if (Mn == -INFINITY) return;
  const float a = (M == -INFINITY) ? 0.f : L * expf(M - Mn);
  const float b = (M2 == -INFINITY) ? 0.f : L2 * expf(M2 - Mn);
  L = a + b;
  M = Mn;
}

// ------------------------------------------------------------------ team layout (per-edge q/k scores)
// T lanes per edge / group (T = H * S, S = dk/VEC lanes per head), 64/T teams per
// wavefront; lane t holds VEC consecutive elements of the att-wide q/k rows and
// ends with its own head's score.  Head leaders (t % S == 0) own the per-head state.
struct Team {
  int T, S;
};

__device__ __forceinline__ int wave_max_int(int v) {
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) v = max(v, __shfl_xor(v, o));
  return v;
}

// Hub groups of the statistics kernels: merge the per-chunk (max, sum-exp)
// partials [slot][2H] (max as fp64, then sum) into m[g,h], rl[g,h] = 1/(sum + 1e-16).
// heavy: int4 {group, first_slot, n_chunks, 0}.  Defined in rhs.hip.
// Merge of long group g's chunk statistics for head h (chunks first .. first+nch-1
// of partials: [slot][M(H) | L(H)]): lanes take strided chunks, then a fixed xor
// tree, so the result does not depend on which wave or launch runs it.
// The stored max is M rounded to fp32 (exact in the fp64 m array and in the
// float records alike) and rl = 1/(sum exp(s - m) + 1e-16) is taken relative to
// that rounded max: L (the sum relative to M) times exp(M - m).  Any shift gives
// the same softmax; this one makes the 16-byte two-head record hold exactly the
// values of the separate arrays.
__device__ __forceinline__ void store_stats(double* __restrict__ m, float* __restrict__ rl, float* __restrict__ mr,
                                            int64_t g, int H, int h, double M, float L) {
  const float m32 = (float)M;
  const double d = M - (double)m32;
  const float Lr = (d == 0.0 || !isfinite(d)) ? L : L * expf((float)d);
  const float r = 1.0f / (Lr + kSoftmaxEps);
  if (m) m[g * H + h] = (double)m32;
  if (rl) rl[g * H + h] = r;
  if (mr) {
    float* rec = mr + g * stats_record_floats(H);
    rec[h] = m32;
    rec[H + h] = r;
  }
}

__device__ __forceinline__ void stats_merge_store(int g, int first, int nch, int H, int h,
                                                  const double* __restrict__ partials, double* __restrict__ m_out,
                                                  float* __restrict__ rl_out, float* __restrict__ mr_out) {
  const int lane = threadIdx.x & 63;
  double M = -INFINITY;
  float L = 0.f;
  for (int c = lane; c < nch; c += kWave)
    online_merge(M, L, partials[(int64_t)(first + c) * 2 * H + h], (float)partials[(int64_t)(first + c) * 2 * H + H + h]);
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) {
    const double M2 = __shfl_xor(M, o);
    const float L2 = __shfl_xor(L, o);
    online_merge(M, L, M2, L2);
  }
  if (lane == 0) store_stats(m_out, rl_out, mr_out, g, H, h, M, L);
}

// Wave-wide (max, sum-exp) of per-lane online states, every head: beyond two heads in
// two phases — the max over the lanes (exact, any order), then the lanes' sums
// rescaled to it (one exp per lane and head) and added in a fixed xor tree — instead
// of a tree of online merges (two exps per merge, six levels, head after head on one
// SIMD: ~6 us of an 8-head long item).  Deterministic; rounding as any fixed tree
// (the per-group kernels agree to 2e-6, tests/test_gpu_parity.py).
template <int MAXH>
__device__ __forceinline__ void lanes_merge(double (&M)[MAXH], float (&L)[MAXH]) {
  if constexpr (MAXH <= 2) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) {
        const double M2 = __shfl_xor(M[h], o);
        const float L2 = __shfl_xor(L[h], o);
        online_merge(M[h], L[h], M2, L2);
      }
  } else {
    double Mx[MAXH];
#pragma unroll
    for (int h = 0; h < MAXH; ++h) Mx[h] = M[h];
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) Mx[h] = fmax(Mx[h], __shfl_xor(Mx[h], o));
#pragma unroll
    for (int h = 0; h < MAXH; ++h) L[h] = M[h] == -INFINITY ? 0.f : L[h] * expf((float)(M[h] - Mx[h]));
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1)
#pragma unroll
      for (int h = 0; h < MAXH; ++h) L[h] += __shfl_xor(L[h], o);
#pragma unroll
    for (int h = 0; h < MAXH; ++h) M[h] = Mx[h];
  }
}

// stats_merge_store for every head at once (MAXH >= H): a lane loads all heads of
// its chunks in one round and the heads' xor trees interleave — the same merges in
// the same order per head, so the same bits.  (A hub group's merge ran head after
// head, a load and a 6-step tree each: serial latency at 8 heads.)
#ifndef GNPDE_MERGE_ALL_HEADS
#define GNPDE_MERGE_ALL_HEADS 1
#endif
template <int MAXH>
__device__ __forceinline__ void stats_merge_store_heads(int g, int first, int nch, int H,
                                                        const double* __restrict__ partials, double* __restrict__ m_out,
                                                        float* __restrict__ rl_out, float* __restrict__ mr_out) {
  if constexpr (!GNPDE_MERGE_ALL_HEADS) {
    for (int h = 0; h < H; ++h) stats_merge_store(g, first, nch, H, h, partials, m_out, rl_out, mr_out);
    return;
  }
  const int lane = threadIdx.x & 63;
  double M[MAXH];
  float L[MAXH];
#pragma unroll
  for (int h = 0; h < MAXH; ++h) {
    M[h] = -INFINITY;
    L[h] = 0.f;
  }
  for (int c = lane; c < nch; c += kWave) {
    const double* __restrict__ p = partials + (int64_t)(first + c) * 2 * H;
    double pm[MAXH], pl[MAXH];
#pragma unroll
    for (int h = 0; h < MAXH; ++h) {
      pm[h] = h < H ? p[h] : -INFINITY;
      pl[h] = h < H ? p[H + h] : 0.0;
    }
#pragma unroll
    for (int h = 0; h < MAXH; ++h)
      if (h < H) online_merge(M[h], L[h], pm[h], (float)pl[h]);
  }
  lanes_merge<MAXH>(M, L);
  if (lane == 0)
#pragma unroll
    for (int h = 0; h < MAXH; ++h)
      if (h < H) store_stats(m_out, rl_out, mr_out, g, H, h, M[h], L[h]);
}

int launch_stats_fixup(const int4* heavy, int64_t n_heavy, int H, const double* partials, double* m, float* rl,
                       float* mr, hipStream_t s);

struct ScoreArgs {
  int mode;
  int H;
  int dk;
  const double* __restrict__ cs;  // [R,H] reference-mode node scores (fp64)
  const float* __restrict__ q;    // [R,ldqk] per-edge modes
  const float* __restrict__ k;
  int64_t ldqk;
  float p0, p1;

  // lane mode: score of edge src->dst, head h, as double (exact for the fp32 modes)
  __device__ __forceinline__ double score(int src, int dst, int h) const {
    if (mode == GNPDE_SCORE_REFERENCE) return cs[(int64_t)src * H + h];
    if (mode == GNPDE_SCORE_UNIFORM) return 0.0;
    return (double)pair_score(mode, q + (int64_t)src * ldqk + h * dk, k + (int64_t)dst * ldqk + h * dk, dk, p0, p1);
  }
};

// sum over the S lanes of a head segment (S a power of two, segments aligned)
__device__ __forceinline__ float seg_sum(float v, int S) {
  for (int o = 1; o < S; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// team mode: lane t (< T) of the team covers elements [t*VEC, t*VEC+VEC) of the
// att-wide rows; returns the score of the lane's head (all S lanes agree).
// Score from the lane's slices already in registers (q of the source, k of
// the destination); the loads are left to the caller so several edges' rows
// can be in flight at once.  The shuffles of seg_sum must run with every lane
// of the wavefront active (callers keep these calls out of divergent code).
template <int VEC>
__device__ __forceinline__ float team_score_regs(const ScoreArgs& sa, const float (&qin)[VEC], const float (&kin)[VEC],
                                                 int S) {
  float q[VEC], k[VEC];
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    q[i] = qin[i];
    k[i] = kin[i];
  }
  const float dk = (float)sa.dk;
  if (sa.mode == GNPDE_SCORE_DOT) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) a = fmaf(q[i], k[i], a);
    return seg_sum(a, S) * rsqrtf(dk);
  }
  if (sa.mode == GNPDE_SCORE_EXP_KERNEL) {
    float a = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const float d = q[i] - k[i];
      a = fmaf(d, d, a);
    }
    a = seg_sum(a, S);
    return sa.p0 * sa.p0 * expf(-(a / (2.0f * sa.p1 * sa.p1)));
  }
  if (sa.mode == GNPDE_SCORE_PEARSON) {
    float sq = 0.f, sk = 0.f;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      sq += q[i];
      sk += k[i];
    }
    const float mq = seg_sum(sq, S) / dk, mk = seg_sum(sk, S) / dk;
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      q[i] -= mq;
      k[i] -= mk;
    }
  }
  float nq = 0.f, nk = 0.f, dot = 0.f;
#pragma unroll
  for (int i = 0; i < VEC; ++i) {
    nq = fmaf(q[i], q[i], nq);
    nk = fmaf(k[i], k[i], nk);
    dot = fmaf(q[i], k[i], dot);
  }
  nq = seg_sum(nq, S);
  nk = seg_sum(nk, S);
  dot = seg_sum(dot, S);
  return dot / (fmaxf(sqrtf(nq), 1e-5f) * fmaxf(sqrtf(nk), 1e-5f));
}

template <int VEC>
__device__ __forceinline__ void team_row(const ScoreArgs& sa, const float* __restrict__ base, int node, int t,
                                         float (&v)[VEC]) {
  load_vec<VEC>(base + (int64_t)node * sa.ldqk + t * VEC, v);
}

template <int VEC>
__device__ __forceinline__ float team_score(const ScoreArgs& sa, int src, int dst, int t, int S) {
  float q[VEC], k[VEC];
  team_row<VEC>(sa, sa.q, src, t, q);
  team_row<VEC>(sa, sa.k, dst, t, k);
  return team_score_regs<VEC>(sa, q, k, S);
}

}  // namespace gnpde
