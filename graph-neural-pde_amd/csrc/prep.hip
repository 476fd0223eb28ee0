// prep.hip — once-per-graph preparation of the ODE blocks' graph
// (ODEblock.reset_graph_data, reference src/base_classes.py:70-90): remaining
// self loops and the random-walk / symmetric (gcn) weight normalisation, with
// the INTENDED semantics the reference's known-answer tests pin
// (test/test_utils.py:111-161, test/test_function_laplacian_diffusion.py:56-86;
// the fork's own batched code crashes or corrupts the edge set).
//
// Everything is deterministic: the loop weight a node keeps is the one of its
// LAST existing loop in COO order (an integer max, not a racing store), and
// every degree is summed sequentially in COO order over the destination- (or
// source-) grouped CSR of gnpde_csr_build — the same fp32 additions, in the
// same order, as torch's CPU scatter_add_ (src/utils.py:191, :230), where the
// device scatter_add_ of the reference would add in atomic arrival order.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace gnpde {

namespace {

int grid_of(int64_t n, int block = 256, int cap = 4096) {
  int64_t g = ceil_div(n, block);
  return (int)(g < 1 ? 1 : (g > cap ? cap : g));
}

size_t align_up(size_t v, size_t a = 256) { return (v + a - 1) / a * a; }

// flags[i] = 1 for a non-loop edge (row != col); the per-batch counts from
// wavefront ballots, kept in a register while the wavefront stays in one batch
// element and added with one integer atomic when it leaves it (and at the end), on a
// grid of at most kFlagBlocks workgroups.  (Round 4 did one atomicAdd per edge on
// counts[b]: 12.4 ms per call at G-arxiv; one per wavefront and step of a 4096-block
// grid: 197 us, still one contended address.)  The grid-stride loop is wavefront-uniform.
constexpr int kFlagBlocks = 256;

__global__ void loop_flags_kernel(const int64_t* __restrict__ ei, int64_t B, int64_t E, int32_t* __restrict__ flags,
                                  unsigned long long* __restrict__ counts) {
  const int64_t n = B * E;
  const int lane = threadIdx.x & 63;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t cur = -1;             // the batch element whose count is held (wavefront-uniform)
  unsigned long long held = 0;
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~63); base < n; base += stride) {
    const int64_t i = base + lane;
    const bool valid = i < n;
    const int64_t b = valid ? (B == 1 ? 0 : i / E) : -1;  // (no 64-bit division for one graph)
    const int64_t e = valid ? i - b * E : 0;
    const bool keep = valid && ei[(b * 2 + 0) * E + e] != ei[(b * 2 + 1) * E + e];
    if (flags && valid) flags[i] = keep;
    // the wavefront's 64 edges span batch elements b0 <= b <= b0 + ceil(64 / E): one ballot each
    const int64_t b0 = B == 1 ? 0 : base / E;
    const int64_t blast = B == 1 ? 0 : (base + 63 < n ? base + 63 : n - 1) / E;
    for (int64_t bb = b0; bb <= blast; ++bb) {
      const unsigned long long m = __ballot(keep && b == bb);
      if (bb != cur) {
        if (lane == 0 && held) atomicAdd(&counts[cur], held);
        cur = bb;
        held = 0;
      }
      held += (unsigned long long)__popcll(m);
    }
  }
  // the workgroup's wavefronts merged in LDS first: one atomic per batch element and
  // workgroup (usually one per workgroup) instead of one per wavefront
  __shared__ long long wb[kBlock / 64];
  __shared__ unsigned long long wc[kBlock / 64];
  const int wv = threadIdx.x >> 6;
  if (lane == 0) {
    wb[wv] = held ? cur : -1;
    wc[wv] = held;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    long long pb = -1;
    unsigned long long pc = 0;
    for (int k = 0; k < kBlock / 64; ++k) {
      if (wb[k] < 0) continue;
      if (wb[k] != pb) {
        if (pc) atomicAdd(&counts[pb], pc);
        pb = wb[k];
        pc = 0;
      }
      pc += wc[k];
    }
    if (pc) atomicAdd(&counts[pb], pc);
  }
}

// the last existing loop of every node: last[b*N + n] = max e with row = col = n
__global__ void last_loop_kernel(const int64_t* __restrict__ ei, int64_t B, int64_t E, int64_t N,
                                 int32_t* __restrict__ last) {
  const int64_t n = B * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / E, e = i - b * E;
    const int64_t r = ei[(b * 2 + 0) * E + e];
    if (r == ei[(b * 2 + 1) * E + e]) atomicMax(&last[b * N + r], (int32_t)e);
  }
}

// non-loop edges keep their COO order (pos = exclusive scan of the flags), then
// one loop per node: out[b, :, K + n] = (n, n), K = non-loop edges per batch
__global__ void emit_loops_kernel(const int64_t* __restrict__ ei, const float* __restrict__ w, int64_t B, int64_t E,
                                  int64_t N, int64_t K, const int32_t* __restrict__ flags,
                                  const int32_t* __restrict__ pos, const int32_t* __restrict__ last, float fill,
                                  int64_t* __restrict__ ei_out, float* __restrict__ w_out) {
  const int64_t E2 = K + N;
  const int64_t n = B * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    if (!flags[i]) continue;
    const int64_t b = i / E, e = i - b * E;
    const int64_t o = pos[i] - b * K;  // position inside batch b
    ei_out[(b * 2 + 0) * E2 + o] = ei[(b * 2 + 0) * E + e];
    ei_out[(b * 2 + 1) * E2 + o] = ei[(b * 2 + 1) * E + e];
    w_out[b * E2 + o] = w ? w[i] : 1.0f;
  }
  for (int64_t j = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; j < B * N; j += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = j / N, v = j - b * N;
    const int32_t l = last[j];
    ei_out[(b * 2 + 0) * E2 + K + v] = v;
    ei_out[(b * 2 + 1) * E2 + K + v] = v;
    w_out[b * E2 + K + v] = l >= 0 ? (w ? w[b * E + l] : 1.0f) : fill;
  }
}

// deg[r] = sum of w over the row's edges, sequentially in COO order (perm of a
// stable grouped CSR), then the normalisation factor of the mode.  A lane sums its
// own row when it has at most kDegLane edges; longer rows (power-law hubs: 7.4k
// edges at G-arxiv) are taken by a wavefront each (degree_long_kernel), 64 weights
// gathered per load and added IN ORDER through readlane — the same sequential fp32
// additions as a lane walking the row (and as torch's CPU scatter_add_), without its
// 7.4k-deep chain of dependent loads (1.58 ms per call at G-arxiv, round 4).
constexpr int kDegLane = 64;
constexpr int kDegUnroll = 16;
constexpr int kDegBatch = 8;

__device__ __forceinline__ float deg_weight(const float* __restrict__ w, const int32_t* __restrict__ perm, int32_t p,
                                            int32_t end) {
  return p < end ? (w ? w[perm[p]] : 1.0f) : 0.0f;
}

__device__ __forceinline__ void store_fac(float* __restrict__ fac, int64_t r, int mode, float d) {
  if (mode == GNPDE_NORM_GCN) {
    const float v = 1.0f / sqrtf(d);  // deg.pow_(-0.5), src/utils.py:192; inf -> 0 (:193)
    fac[r] = isinf(v) ? 0.f : v;
  } else {
    fac[r] = 1.0f / d;  // deg.pow_(-1), src/utils.py:231
  }
}

__global__ void degree_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm, int64_t R,
                              const float* __restrict__ w, int mode, float* __restrict__ fac) {
  const int lane = threadIdx.x & 63;
  const int64_t r0 = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x - lane);  // the wavefront's first row
  if (r0 >= R) return;  // wavefront-uniform
  const int64_t r = r0 + lane;
  const bool valid = r < R;
  const int32_t b = valid ? rowptr[r] : 0, e = valid ? rowptr[r + 1] : 0;
  const bool longr = e - b > kDegLane;
  if (!valid || longr) return;  // long rows: degree_long_kernel
  float d = 0.f;
  if (!w) {
    d = (float)(e - b);  // unit weights: the in-order sum of at most 64 ones
  } else {
    // kDegBatch positions' perm entries, then their weights, in flight at once; the adds
    // stay in COO order (the chain of dependent loads was the cost: 32 us at G-arxiv)
    for (int32_t p0 = b; p0 < e; p0 += kDegBatch) {
      int32_t q[kDegBatch];
#pragma unroll
      for (int k = 0; k < kDegBatch; ++k) q[k] = p0 + k < e ? perm[p0 + k] : -1;
      float v[kDegBatch];
#pragma unroll
      for (int k = 0; k < kDegBatch; ++k) v[k] = q[k] >= 0 ? w[q[k]] : 0.f;
#pragma unroll
      for (int k = 0; k < kDegBatch; ++k)
        if (p0 + k < e) d += v[k];
    }
  }
  store_fac(fac, r, mode, d);
}

// The rows longer than kDegLane edges, one wavefront per row (in one wavefront the
// hub rows of a 64-row block — RMAT puts them together at low ids — were summed one
// after another: 1.56 ms per call at G-arxiv).  The wave's 64 weights per load are
// added in order through readlane (the sequential sum), the next chunk in flight.
__global__ void degree_long_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm, int64_t R,
                                   const float* __restrict__ w, int mode, float* __restrict__ fac) {
  const int lane = threadIdx.x & 63;
  const int64_t r = (int64_t)blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6);
  if (r >= R) return;
  const int32_t bb = rowptr[r], ee = rowptr[r + 1];
  if (ee - bb <= kDegLane) return;  // wavefront-uniform: degree_kernel's lanes took it
  // Integral weights whose |w| sum stays below 2^24 (unit weights: any row shorter than
  // 2^24): every partial sum in ANY order is an exactly representable integer, so lane-
  // strided sums and a tree give the sequential sum's bits.  kDegUnroll loads per lane in
  // flight (perm, then the weights); the fp32 sum of |w| is monotone in its addends, so
  // it reaches 2^24 exactly when the true sum does.
  {
    float s = 0.f, a = 0.f;
    bool ok = true;
    for (int32_t p0 = bb; p0 < ee; p0 += 64 * kDegUnroll) {
      int32_t q[kDegUnroll];
#pragma unroll
      for (int k = 0; k < kDegUnroll; ++k) {
        const int32_t p = p0 + k * 64 + lane;
        q[k] = p < ee ? (w ? perm[p] : 0) : -1;
      }
#pragma unroll
      for (int k = 0; k < kDegUnroll; ++k) {
        const float v = q[k] < 0 ? 0.f : (w ? w[q[k]] : 1.0f);
        s += v;
        a += fabsf(v);
        ok = ok && v == rintf(v);
      }
    }
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) {
      s += __shfl_xor(s, off);
      a += __shfl_xor(a, off);
    }
    if (__ballot(!ok) == 0 && a < 16777216.0f) {  // wavefront-uniform (a is lane-equal after the tree)
      if (lane == 0) store_fac(fac, r, mode, s);
      return;
    }
  }
  float acc = 0.f;
  float v = deg_weight(w, perm, bb + lane, ee);
  for (int32_t p0 = bb; p0 < ee; p0 += 64) {
    const float nv = deg_weight(w, perm, p0 + 64 + lane, ee);  // the next chunk, in flight
    const int cnt = ee - p0 < 64 ? ee - p0 : 64;
    if (cnt == 64) {
      // whole chunks: constant lane indices, no loop counter between the dependent adds
      // (a counted readlane loop cost ~120 cycles per edge: 370 us for G-arxiv's hubs)
#pragma unroll
      for (int k = 0; k < 64; ++k) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
    } else {
      for (int k = 0; k < cnt; ++k) acc += __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), k));
    }
    v = nv;
  }
  if (lane == 0) store_fac(fac, r, mode, acc);
}

__global__ void scale_kernel(const int64_t* __restrict__ ei, const float* __restrict__ w, int64_t B, int64_t E,
                             int64_t N, int mode, const float* __restrict__ fac, float* __restrict__ w_out) {
  const int64_t n = B * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / E, e = i - b * E;
    const int64_t r = b * N + ei[(b * 2 + 0) * E + e];
    const int64_t c = b * N + ei[(b * 2 + 1) * E + e];
    const float wv = w ? w[i] : 1.0f;
    float o;
    if (mode == GNPDE_NORM_RW_ROW)
      o = fac[r] * wv;  // deg_inv[row] * w (norm_dim 0, src/utils.py:232)
    else if (mode == GNPDE_NORM_RW_COL)
      o = wv * fac[c];  // w * deg_inv[col] (norm_dim 1)
    else
      o = fac[r] * wv * fac[c];  // deg^-1/2[row] * w * deg^-1/2[col] (src/utils.py:194)
    w_out[i] = o;
  }
}

}  // namespace
}  // namespace gnpde

using namespace gnpde;

extern "C" {

size_t gnpde_self_loops_workspace_bytes(int64_t B, int64_t E, int64_t N) {
  const int64_t n = B * E > 0 ? B * E : 1;
  size_t scan = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, scan, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return 2 * align_up(sizeof(int32_t) * (size_t)n) + align_up(sizeof(int32_t) * (size_t)(B * N)) +
         align_up(sizeof(unsigned long long) * (size_t)B) + align_up(scan);
}

int gnpde_self_loops_count(const int64_t* edge_index, int64_t B, int64_t E, int64_t* nonloop, void* workspace,
                           size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(B >= 1 && E >= 0, GNPDE_EINVAL, "self_loops_count: bad sizes");
  GNPDE_REQUIRE(nonloop && workspace, GNPDE_EINVAL, "self_loops_count: NULL pointer");
  GNPDE_REQUIRE(workspace_bytes >= align_up(sizeof(unsigned long long) * (size_t)B), GNPDE_EINVAL,
                "self_loops_count: workspace too small");
  hipStream_t s = as_stream(stream);
  auto* counts = static_cast<unsigned long long*>(workspace);
  GNPDE_HIP(hipMemsetAsync(counts, 0, sizeof(unsigned long long) * B, s));
  if (B * E > 0) {
    GNPDE_REQUIRE(edge_index != nullptr, GNPDE_EINVAL, "self_loops_count: NULL edge_index");
    loop_flags_kernel<<<grid_of(B * E, 256, kFlagBlocks), 256, 0, s>>>(edge_index, B, E, nullptr, counts);
    GNPDE_LAUNCH_CHECK();
  }
  GNPDE_HIP(hipMemcpyAsync(nonloop, counts, sizeof(unsigned long long) * B, hipMemcpyDeviceToHost, s));
  GNPDE_HIP(hipStreamSynchronize(s));
  return GNPDE_OK;
}

int gnpde_add_self_loops(const int64_t* edge_index, const float* w, int64_t B, int64_t E, int64_t N, float fill,
                         int64_t K, int64_t* ei_out, float* w_out, void* workspace, size_t workspace_bytes,
                         void* stream) {
  GNPDE_REQUIRE(B >= 1 && E >= 0 && N >= 1 && K >= 0 && K <= E, GNPDE_EINVAL, "add_self_loops: bad sizes");
  GNPDE_REQUIRE(B * E < (int64_t)INT32_MAX && B * N < (int64_t)INT32_MAX, GNPDE_EUNSUPPORTED,
                "add_self_loops: B*E and B*N must fit int32");
  GNPDE_REQUIRE(ei_out && w_out && workspace, GNPDE_EINVAL, "add_self_loops: NULL pointer");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_self_loops_workspace_bytes(B, E, N), GNPDE_EINVAL,
                "add_self_loops: workspace too small");
  hipStream_t s = as_stream(stream);
  const int64_t n = B * E > 0 ? B * E : 1;
  char* ws = static_cast<char*>(workspace);
  const size_t a = align_up(sizeof(int32_t) * (size_t)n);
  int32_t* flags = reinterpret_cast<int32_t*>(ws);
  int32_t* pos = reinterpret_cast<int32_t*>(ws + a);
  int32_t* last = reinterpret_cast<int32_t*>(ws + 2 * a);
  auto* counts = reinterpret_cast<unsigned long long*>(ws + 2 * a + align_up(sizeof(int32_t) * (size_t)(B * N)));
  void* tmp = reinterpret_cast<char*>(counts) + align_up(sizeof(unsigned long long) * (size_t)B);
  size_t tmp_bytes = workspace_bytes - (size_t)(static_cast<char*>(tmp) - ws);
  GNPDE_HIP(hipMemsetAsync(last, 0xff, sizeof(int32_t) * B * N, s));  // -1: no existing loop
  GNPDE_HIP(hipMemsetAsync(counts, 0, sizeof(unsigned long long) * B, s));
  if (B * E > 0) {
    GNPDE_REQUIRE(edge_index != nullptr, GNPDE_EINVAL, "add_self_loops: NULL edge_index");
    loop_flags_kernel<<<grid_of(B * E, 256, kFlagBlocks), 256, 0, s>>>(edge_index, B, E, flags, counts);
    GNPDE_LAUNCH_CHECK();
    last_loop_kernel<<<grid_of(B * E), 256, 0, s>>>(edge_index, B, E, N, last);
    GNPDE_LAUNCH_CHECK();
    GNPDE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, flags, pos, (int)(B * E), s));
  }
  emit_loops_kernel<<<grid_of(B * (E > N ? E : N)), 256, 0, s>>>(edge_index, w, B, E, N, K, flags, pos, last, fill,
                                                                  ei_out, w_out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_norm_weights_f32(const int64_t* edge_index, const float* w, int64_t B, int64_t E, int64_t N,
                           const int32_t* rowptr, const int32_t* perm, int mode, float* fac, float* w_out,
                           void* stream) {
  GNPDE_REQUIRE(B >= 1 && E >= 0 && N >= 1, GNPDE_EINVAL, "norm_weights: bad sizes");
  GNPDE_REQUIRE(mode == GNPDE_NORM_RW_ROW || mode == GNPDE_NORM_RW_COL || mode == GNPDE_NORM_GCN, GNPDE_EINVAL,
                "norm_weights: unknown mode %d", mode);
  GNPDE_REQUIRE(rowptr && fac && (E == 0 || (edge_index && perm && w_out)), GNPDE_EINVAL,
                "norm_weights: NULL pointer");
  hipStream_t s = as_stream(stream);
  degree_kernel<<<(unsigned)ceil_div(B * N, 256), 256, 0, s>>>(rowptr, perm, B * N, w, mode, fac);
  GNPDE_LAUNCH_CHECK();
  degree_long_kernel<<<(unsigned)ceil_div(B * N, (int64_t)kWavesPerBlock), 256, 0, s>>>(rowptr, perm, B * N, w, mode,
                                                                                        fac);
  GNPDE_LAUNCH_CHECK();
  if (B * E > 0) {
    scale_kernel<<<grid_of(B * E), 256, 0, s>>>(edge_index, w, B, E, N, mode, fac, w_out);
    GNPDE_LAUNCH_CHECK();
  }
  return GNPDE_OK;
}

}  // extern "C"
