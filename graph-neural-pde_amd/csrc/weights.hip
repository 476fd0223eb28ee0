// weights.hip — edge-weight producers of the mixed and hard-attention ODE blocks.
//
// Both blocks integrate the same Laplacian RHS (K1) as the constant block; they
// differ only in where its edge weights come from, once per forward:
//   * MixedODEblock.get_mixed_attention   src/block_mixed.py:29-33
//       w = mean_h(att) * (1 - sigmoid(gamma)) + edge_weight * sigmoid(gamma)
//   * HardAttODEblock.forward             src/block_transformer_hard_attention.py:37-60
//       eval : w = mean_h(att)
//       train: keep edges whose mean attention exceeds the (1 - att_samp_pct)
//              quantile, then renormalise per softmax group (:32-35).
// All three are short elementwise / per-group passes over E weights.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace gnpde {

// out[i] = mean_h att[i*H + h]  [ * (1 - s) + ew[i] * s,  s = sigmoid(*gamma) ]
__global__ void mix_weights_kernel(const float* __restrict__ att, int H, const float* __restrict__ ew,
                                   const float* __restrict__ gamma, int64_t n, float* __restrict__ out) {
  float s = 0.f;
  if (gamma) s = 1.f / (1.f + expf(-gamma[0]));  // torch.sigmoid in fp32
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    float m;
    if (H == 1) {
      m = att[i];
    } else {
      float a = 0.f;
      for (int h = 0; h < H; ++h) a += att[i * H + h];
      m = a / (float)H;  // attention.mean(dim=2), fp32
    }
    out[i] = gamma ? m * (1.f - s) + ew[i] * s : m;
  }
}

// Group renormalisation in two passes over the grouped (CSR-order) positions:
// group_gather_kernel: t[p] = w_in[perm[p]] (position-parallel: the COO-order weights
// brought into group order once, so no group walks a perm -> w chain of dependent
// loads); group_normalize_kernel: one wavefront per group sums its contiguous run of
// t in a fixed order (lane-strided partial sums, UNR loads in flight per lane, then a
// butterfly) and writes w_out[perm[p]] = t[p] / (sum + 1e-16).  (Round 5 walked
// w_in[perm[p]] per group: the 7.4k-edge hub group of G-arxiv was a chain of ~230
// dependent loads, 342 us per training forward.)
__global__ void group_gather_kernel(const int32_t* __restrict__ perm, int64_t nnz, const float* __restrict__ w_in,
                                    float* __restrict__ t) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += stride) t[p] = w_in[perm[p]];
}

__global__ void group_normalize_kernel(const int32_t* __restrict__ rowptr, const int32_t* __restrict__ perm,
                                       int64_t R, const float* __restrict__ t, float* __restrict__ w_out) {
  constexpr int UNR = 4;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t wave = (blockIdx.x * (int64_t)blockDim.x + threadIdx.x) / kWave;
  const int64_t nwaves = (int64_t)gridDim.x * blockDim.x / kWave;
  for (int64_t r = wave; r < R; r += nwaves) {
    const int b = rowptr[r], e = rowptr[r + 1];
    float s = 0.f;
    for (int p0 = b; p0 < e; p0 += UNR * kWave) {
      float v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int p = p0 + u * kWave + lane;
        v[u] = p < e ? t[p] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u) s += v[u];
    }
    s = wave_sum(s);
    const float den = s + kSoftmaxEps;
    for (int p0 = b; p0 < e; p0 += UNR * kWave) {
      int idx[UNR];
      float v[UNR];
#pragma unroll
      for (int u = 0; u < UNR; ++u) {
        const int p = p0 + u * kWave + lane;
        idx[u] = p < e ? perm[p] : -1;
        v[u] = p < e ? t[p] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < UNR; ++u)
        if (idx[u] >= 0) w_out[idx[u]] = v[u] / den;
    }
  }
}

// The hard-attention sampling mask as weights over the FULL graph
// (src/block_transformer_hard_attention.py:52-55): out[i] = v[i] if v[i] > *thr
// else 0, and *count = the retained edges (one atomic per wavefront).  Zero-weight
// edges add exact zeros to every row sum and group sum, so the RHS over the full
// graph with these weights equals the RHS over the compacted edge list — without
// building a new CSR / plan for every training forward.
constexpr int kMaskBlocks = 256;  // the mask's grid: one per CU, each streaming its share

__global__ void threshold_mask_kernel(const float* __restrict__ v, int64_t n, const float* __restrict__ thr,
                                      float* __restrict__ out, unsigned long long* __restrict__ count) {
  const float t = *thr;
  const int lane = threadIdx.x & (kWave - 1);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  unsigned long long kept = 0;
  for (int64_t base = blockIdx.x * (int64_t)blockDim.x + (threadIdx.x & ~(kWave - 1)); base < n; base += stride) {
    const int64_t i = base + lane;
    const bool live = i < n;
    const float x = live ? v[i] : 0.f;
    const bool keep = live && x > t;
    if (live) out[i] = keep ? x : 0.f;
    kept += __popcll(__ballot(keep));
  }
  // one atomic per workgroup on a grid of at most kMaskBlocks (one per wavefront on a
  // 4096-workgroup grid was 16k atomics on one address: 199 us for G-arxiv's 1.2M edges)
  __shared__ unsigned long long wk[kWavesPerBlock];
  if (lane == 0) wk[threadIdx.x >> 6] = kept;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned long long t = 0;
    for (int w = 0; w < kWavesPerBlock; ++w) t += wk[w];
    if (t) atomicAdd(count, t);
  }
}

// The sampled graph of hard attention in the plan's own structure: every work item
// (row, edge_begin, edge_end, slot) keeps its row, slot and edge_begin, and its
// edges with a nonzero weight are moved to the front of its range in their order
// (a stable partition by ballot), edge_end shrinking to edge_begin + the kept count.
// The aggregation then gathers only retained edges, in the order and hub chunks of
// the full plan: the same sums as over the masked full graph (a dropped edge added
// an exact 0), no plan rebuild and no host read.  Four items per wavefront (16-lane
// slots; the plan's items are stored longest first, so a wave's items have similar
// lengths): 35 -> ~10 us for G-arxiv's 170k items.
constexpr int kCompactSL = 16;

__global__ __launch_bounds__(256) void compact_items_kernel(const int4* __restrict__ items, int n_items,
                                                            const int* __restrict__ col, const float* __restrict__ w,
                                                            int* __restrict__ col_out, float* __restrict__ w_out,
                                                            int4* __restrict__ items_out) {
  constexpr int SPW = kWave / kCompactSL;
  const int lane = threadIdx.x & (kWave - 1);
  const int slot = lane / kCompactSL, sl = lane % kCompactSL;
  const int item = (blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)) * SPW + slot;
  const bool live = item < n_items;
  const int4 it = live ? items[item] : make_int4(0, 0, 0, 0);
  const int len = it.z - it.y;
  int maxlen = len;
#pragma unroll
  for (int o = 1; o < kWave; o <<= 1) maxlen = max(maxlen, __shfl_xor(maxlen, o));
  int kept = 0;
  for (int j = 0; j < maxlen; j += kCompactSL) {  // wave-uniform trip count
    const int p = it.y + j + sl;
    const bool in = j + sl < len;
    const float v = in ? w[p] : 0.f;
    const int c = in ? col[p] : 0;
    const bool keep = in && v != 0.f;
    const unsigned long long m = (__ballot(keep) >> (slot * kCompactSL)) & 0xffffull;
    const int before = __popcll(m & ((1ull << sl) - 1ull));
    if (keep) {
      col_out[it.y + kept + before] = c;
      w_out[it.y + kept + before] = v;
    }
    kept += __popcll(m);
  }
  if (live && sl == 0) items_out[item] = make_int4(it.x, it.y, it.y + kept, it.w);
}

// torch.quantile(v, q) (linear interpolation) on a sorted copy:
// rank = q*(n-1) in fp32, lo = floor, hi = ceil, w = rank - lo,
// lerp(a, b, w) = w < 0.5 ? a + w (b - a) : b - (b - a)(1 - w)   (ATen's lerp).
// No FMA contraction here: the threshold must equal torch.quantile bit for bit
// (the sampling mask is a strict comparison against it).
__global__ void quantile_pick_kernel(const float* __restrict__ sorted, int64_t n, float q, float* __restrict__ out) {
#pragma clang fp contract(off)
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  const float rank = q * (float)(n - 1);
  int64_t lo = (int64_t)rank;
  int64_t hi = (int64_t)ceilf(rank);
  if (lo < 0) lo = 0;
  if (hi > n - 1) hi = n - 1;
  if (lo > n - 1) lo = n - 1;
  const float w = rank - (float)lo;
  const float a = sorted[lo], b = sorted[hi];
  out[0] = (fabsf(w) < 0.5f) ? a + w * (b - a) : b - (b - a) * (1.f - w);
}

static int grid_for_n(int64_t n, int block = 256, int cap = 4096) {
  int64_t g = ceil_div(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

static size_t align_up256(size_t v) { return (v + 255) / 256 * 256; }

static size_t sort_keys_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortKeys(nullptr, bytes, (const float*)nullptr, (float*)nullptr, (int)n);
  return bytes;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_mix_weights_f32(const float* att, int H, const float* ew, const float* gamma, int64_t n, float* out,
                          void* stream) {
  GNPDE_REQUIRE(H >= 1 && n >= 0, GNPDE_EINVAL, "mix_weights: bad sizes H=%d n=%lld", H, (long long)n);
  GNPDE_REQUIRE((gamma == nullptr) == (ew == nullptr), GNPDE_EINVAL,
                "mix_weights: gamma and edge_weight must both be set or both be NULL");
  if (n == 0) return GNPDE_OK;
  GNPDE_REQUIRE(att && out, GNPDE_EINVAL, "mix_weights: NULL pointer");
  mix_weights_kernel<<<grid_for_n(n), 256, 0, as_stream(stream)>>>(att, H, ew, gamma, n, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

size_t gnpde_group_normalize_workspace_bytes(int64_t nnz) { return sizeof(float) * (size_t)(nnz > 0 ? nnz : 1); }

int gnpde_group_normalize_f32(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, const float* w_in,
                              float* w_out, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(R >= 1 && nnz >= 0, GNPDE_EINVAL, "group_normalize: bad sizes");
  GNPDE_REQUIRE(w_in != w_out, GNPDE_EINVAL, "group_normalize: in-place is not supported");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowptr && perm && w_in && w_out && workspace, GNPDE_EINVAL, "group_normalize: NULL pointer");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_group_normalize_workspace_bytes(nnz), GNPDE_EINVAL,
                "group_normalize: workspace too small");
  hipStream_t s = as_stream(stream);
  float* t = static_cast<float*>(workspace);
  const int64_t gblocks = ceil_div(nnz, (int64_t)kBlock);
  group_gather_kernel<<<(int)(gblocks < 4096 ? gblocks : 4096), kBlock, 0, s>>>(perm, nnz, w_in, t);
  GNPDE_LAUNCH_CHECK();
  const int64_t blocks = ceil_div(R, (int64_t)kWavesPerBlock);
  group_normalize_kernel<<<(int)(blocks < 65536 ? blocks : 65536), kBlock, 0, s>>>(rowptr, perm, R, t, w_out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_threshold_mask_f32(const float* v, int64_t n, const float* thr, float* out, int64_t* count, void* stream) {
  GNPDE_REQUIRE(n >= 0 && thr && count && (n == 0 || (v && out)), GNPDE_EINVAL, "threshold_mask: bad arguments");
  hipStream_t s = as_stream(stream);
  GNPDE_HIP(hipMemsetAsync(count, 0, sizeof(int64_t), s));
  if (n == 0) return GNPDE_OK;
  const int64_t blocks = ceil_div(n, kBlock);
  threshold_mask_kernel<<<(int)(blocks < kMaskBlocks ? blocks : kMaskBlocks), kBlock, 0, s>>>(
      v, n, thr, out, reinterpret_cast<unsigned long long*>(count));
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_compact_items_f32(const int32_t* items, int64_t n_items, const int32_t* col, const float* w,
                            int32_t* col_out, float* w_out, int32_t* items_out, void* stream) {
  GNPDE_REQUIRE(n_items >= 0 && n_items < INT32_MAX && (n_items == 0 || (items && col && w && col_out && w_out &&
                items_out)), GNPDE_EINVAL, "compact_items: bad arguments");
  GNPDE_REQUIRE(items_out != items && col_out != col && w_out != w, GNPDE_EINVAL,
                "compact_items: outputs may not alias the inputs");
  if (n_items == 0) return GNPDE_OK;
  const unsigned grid = (unsigned)ceil_div(n_items, (int64_t)kWavesPerBlock * (kWave / kCompactSL));
  compact_items_kernel<<<grid, kBlock, 0, as_stream(stream)>>>(reinterpret_cast<const int4*>(items), (int)n_items,
                                                                col, w, col_out, w_out,
                                                                reinterpret_cast<int4*>(items_out));
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

size_t gnpde_quantile_workspace_bytes(int64_t n) {
  const int64_t m = n > 0 ? n : 1;
  return align_up256(sizeof(float) * (size_t)m) + align_up256(sort_keys_bytes(m));
}

int gnpde_quantile_f32(const float* v, int64_t n, double q, float* out, void* workspace, size_t workspace_bytes,
                       void* stream) {
  GNPDE_REQUIRE(n >= 1 && n < (int64_t)INT32_MAX, GNPDE_EINVAL, "quantile: n=%lld out of range", (long long)n);
  GNPDE_REQUIRE(q >= 0.0 && q <= 1.0, GNPDE_EINVAL, "quantile: q=%g outside [0, 1]", q);
  GNPDE_REQUIRE(v && out && workspace, GNPDE_EINVAL, "quantile: NULL pointer");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_quantile_workspace_bytes(n), GNPDE_EINVAL, "quantile: workspace too small");
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  float* sorted = reinterpret_cast<float*>(ws);
  const size_t a = align_up256(sizeof(float) * (size_t)n);
  size_t tmp_bytes = workspace_bytes - a;
  GNPDE_HIP(hipcub::DeviceRadixSort::SortKeys(ws + a, tmp_bytes, v, sorted, (int)n, 0, 32, s));
  quantile_pick_kernel<<<1, 64, 0, s>>>(sorted, n, (float)q, out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
