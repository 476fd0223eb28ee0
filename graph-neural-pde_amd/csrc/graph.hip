// graph.hip — once-per-graph preparation: COO -> block-diagonal CSR/CSC, weight
// permutation, in-degrees and the hub-splitting work plan.
//
// The reference rebuilds a [B,N,N] dense adjacency on every RHS call
// (src/function_laplacian_diffusion.py:41-57).  Here the graph is turned into
// an int32 CSR once (stable radix sort, so in-row order = COO order) and every
// RHS evaluation reuses it.
#include <hipcub/hipcub.hpp>

#include <cstdarg>
#include <mutex>

#include "common.hpp"

namespace gnpde {

static thread_local std::string g_last_error;

void set_error(const char* fmt, ...) {
  char buf[1024];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof(buf), fmt, ap);
  va_end(ap);
  g_last_error = buf;
}

// keys[i] = b*N + edge_index[b, key_row, e], vals[i] = i (= b*E + e)
__global__ void make_keys_kernel(const int64_t* __restrict__ ei, int64_t B, int64_t E, int64_t N, int key_row,
                                 int32_t* __restrict__ keys, int32_t* __restrict__ vals) {
  const int64_t n = B * E;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x) {
    const int64_t b = i / E, e = i - b * E;
    keys[i] = (int32_t)(b * N + ei[(b * 2 + key_row) * E + e]);
    vals[i] = (int32_t)i;
  }
}

// rowptr[r] = lower_bound(sorted_keys, r), r in [0, R]
__global__ void rowptr_kernel(const int32_t* __restrict__ sk, int64_t nnz, int64_t R, int32_t* __restrict__ rowptr) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r <= R; r += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = nnz;
    while (lo < hi) {
      const int64_t mid = (lo + hi) >> 1;
      if (sk[mid] < r) lo = mid + 1; else hi = mid;
    }
    rowptr[r] = (int32_t)lo;
  }
}

// col[p] = b*N + edge_index[b, 1-key_row, e] for e = perm[p]
__global__ void col_kernel(const int64_t* __restrict__ ei, const int32_t* __restrict__ perm, int64_t nnz, int64_t E,
                           int64_t N, int other_row, int32_t* __restrict__ col) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = perm[p];
    const int64_t b = i / E, e = i - b * E;
    col[p] = (int32_t)(b * N + ei[(b * 2 + other_row) * E + e]);
  }
}

__global__ void gather_weights_kernel(const float* __restrict__ w, int64_t nnz, int H, const int32_t* __restrict__ perm,
                                      float* __restrict__ out) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
    const int64_t i = perm[p];
    if (H == 1) {
      out[p] = w[i];
    } else {
      // attention_weights.mean(dim=2) in fp32 (function_laplacian_diffusion.py:46)
      float s = 0.f;
      for (int h = 0; h < H; ++h) s += w[i * H + h];
      out[p] = s / (float)H;
    }
  }
}

// rowidx[p] = r such that rowptr[r] <= p < rowptr[r+1]  (upper_bound - 1)
__global__ void rowidx_kernel(const int32_t* __restrict__ rowptr, int64_t R, int64_t nnz, int32_t* __restrict__ rowidx) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < nnz; p += (int64_t)gridDim.x * blockDim.x) {
    int64_t lo = 0, hi = R;  // find last r with rowptr[r] <= p
    while (lo < hi) {
      const int64_t mid = (lo + hi + 1) >> 1;
      if (rowptr[mid] <= p) lo = mid; else hi = mid - 1;
    }
    rowidx[p] = (int32_t)lo;
  }
}

__global__ void count_kernel(const int32_t* __restrict__ idx, int64_t n, int32_t* __restrict__ cnt) {
  for (int64_t p = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; p < n; p += (int64_t)gridDim.x * blockDim.x)
    atomicAdd(&cnt[idx[p]], 1);
}

// ---- plan: per-row chunk counts, then item/heavy emission
__global__ void plan_count_kernel(const int32_t* __restrict__ rowptr, int64_t R, int32_t chunk,
                                  int32_t* __restrict__ n_it, int32_t* __restrict__ n_sl,
                                  int32_t* __restrict__ n_hv) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t deg = rowptr[r + 1] - rowptr[r];
    const bool heavy = deg > chunk;
    const int32_t nch = heavy ? (deg + chunk - 1) / chunk : 1;
    n_it[r] = nch;
    n_sl[r] = heavy ? nch : 0;
    n_hv[r] = heavy ? 1 : 0;
  }
}

__global__ void plan_emit_kernel(const int32_t* __restrict__ rowptr, int64_t R, const int32_t* __restrict__ o_it,
                                 const int32_t* __restrict__ o_sl, const int32_t* __restrict__ o_hv,
                                 const int32_t* __restrict__ n_it, int4* __restrict__ items,
                                 int4* __restrict__ heavy) {
  for (int64_t r = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; r < R; r += (int64_t)gridDim.x * blockDim.x) {
    const int32_t beg = rowptr[r], end = rowptr[r + 1];
    const int32_t nch = n_it[r];
    if (nch == 1) {  // deg <= chunk: the item owns its row
      items[o_it[r]] = make_int4((int)r, beg, end, -1);
      continue;
    }
    const int32_t deg = end - beg;
    const int32_t per = (deg + nch - 1) / nch;
    for (int32_t c = 0; c < nch; ++c) {
      const int32_t b0 = beg + c * per;
      const int32_t b1 = min(end, b0 + per);
      items[o_it[r] + c] = make_int4((int)r, b0, b1, o_sl[r] + c);
    }
    heavy[o_hv[r]] = make_int4((int)r, o_sl[r], nch, 0);
  }
}

static int grid_for(int64_t n, int block = 256, int cap = 4096) {
  int64_t g = ceil_div(n, block);
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

}  // namespace gnpde

using namespace gnpde;

extern "C" {

int gnpde_abi_version(void) { return GNPDE_ABI_VERSION; }

const char* gnpde_last_error(void) { return g_last_error.c_str(); }

static size_t cub_sort_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr,
                                     (const int32_t*)nullptr, (int32_t*)nullptr, (int)n, 0, 32);
  return bytes;
}

static size_t align_up(size_t v, size_t a = 256) { return (v + a - 1) / a * a; }

size_t gnpde_csr_workspace_bytes(int64_t B, int64_t E, int64_t N) {
  (void)N;
  const int64_t n = B * E;
  return 3 * align_up(sizeof(int32_t) * (size_t)(n > 0 ? n : 1)) + align_up(cub_sort_bytes(n > 0 ? n : 1));
}

int gnpde_csr_build(const int64_t* edge_index, int64_t B, int64_t E, int64_t N, int key_row, int32_t* rowptr,
                    int32_t* col, int32_t* perm, void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(B >= 1 && E >= 0 && N >= 1, GNPDE_EINVAL, "csr_build: bad sizes B=%lld E=%lld N=%lld",
                (long long)B, (long long)E, (long long)N);
  GNPDE_REQUIRE(key_row == 0 || key_row == 1, GNPDE_EINVAL, "csr_build: key_row must be 0 or 1");
  GNPDE_REQUIRE(B * N < (int64_t)INT32_MAX && B * E < (int64_t)INT32_MAX, GNPDE_EUNSUPPORTED,
                "csr_build: B*N and B*E must fit int32");
  GNPDE_REQUIRE(rowptr != nullptr, GNPDE_EINVAL, "csr_build: rowptr is NULL");
  const int64_t nnz = B * E, R = B * N;
  hipStream_t s = as_stream(stream);
  if (nnz == 0) {
    GNPDE_HIP(hipMemsetAsync(rowptr, 0, sizeof(int32_t) * (R + 1), s));
    return GNPDE_OK;
  }
  GNPDE_REQUIRE(edge_index && col && perm && workspace, GNPDE_EINVAL, "csr_build: NULL pointer");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_csr_workspace_bytes(B, E, N), GNPDE_EINVAL,
                "csr_build: workspace too small (%zu < %zu)", workspace_bytes, gnpde_csr_workspace_bytes(B, E, N));
  char* ws = static_cast<char*>(workspace);
  const size_t a = align_up(sizeof(int32_t) * (size_t)nnz);
  int32_t* keys_in = reinterpret_cast<int32_t*>(ws);
  int32_t* keys_out = reinterpret_cast<int32_t*>(ws + a);
  int32_t* vals_in = reinterpret_cast<int32_t*>(ws + 2 * a);
  void* tmp = ws + 3 * a;
  size_t tmp_bytes = workspace_bytes - 3 * a;
  int end_bit = 1;
  while (end_bit < 31 && ((int64_t)1 << end_bit) <= R) ++end_bit;

  make_keys_kernel<<<grid_for(nnz), 256, 0, s>>>(edge_index, B, E, N, key_row, keys_in, vals_in);
  GNPDE_LAUNCH_CHECK();
  GNPDE_HIP(hipcub::DeviceRadixSort::SortPairs(tmp, tmp_bytes, keys_in, keys_out, vals_in, perm, (int)nnz, 0,
                                               end_bit, s));
  rowptr_kernel<<<grid_for(R + 1), 256, 0, s>>>(keys_out, nnz, R, rowptr);
  GNPDE_LAUNCH_CHECK();
  col_kernel<<<grid_for(nnz), 256, 0, s>>>(edge_index, perm, nnz, E, N, 1 - key_row, col);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_gather_weights_f32(const float* w_in, int64_t nnz, int H, const int32_t* perm, float* w_out,
                             void* stream) {
  GNPDE_REQUIRE(H >= 1, GNPDE_EINVAL, "gather_weights: H must be >= 1");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(w_in && perm && w_out, GNPDE_EINVAL, "gather_weights: NULL pointer");
  gather_weights_kernel<<<grid_for(nnz), 256, 0, as_stream(stream)>>>(w_in, nnz, H, perm, w_out);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_csr_rowidx(const int32_t* rowptr, int64_t R, int64_t nnz, int32_t* rowidx, void* stream) {
  GNPDE_REQUIRE(R >= 1 && nnz >= 0, GNPDE_EINVAL, "csr_rowidx: bad sizes");
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(rowptr && rowidx, GNPDE_EINVAL, "csr_rowidx: NULL pointer");
  rowidx_kernel<<<grid_for(nnz), 256, 0, as_stream(stream)>>>(rowptr, R, nnz, rowidx);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

int gnpde_indegree_i32(const int32_t* idx, int64_t nnz, int64_t R, int32_t* deg, void* stream) {
  GNPDE_REQUIRE(deg != nullptr && R >= 1, GNPDE_EINVAL, "indegree: bad args");
  hipStream_t s = as_stream(stream);
  GNPDE_HIP(hipMemsetAsync(deg, 0, sizeof(int32_t) * R, s));
  if (nnz == 0) return GNPDE_OK;
  GNPDE_REQUIRE(idx != nullptr, GNPDE_EINVAL, "indegree: NULL idx");
  count_kernel<<<grid_for(nnz), 256, 0, s>>>(idx, nnz, deg);
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

static size_t cub_scan_bytes(int64_t n) {
  size_t bytes = 0;
  (void)hipcub::DeviceScan::ExclusiveSum(nullptr, bytes, (const int32_t*)nullptr, (int32_t*)nullptr, (int)n);
  return bytes;
}

size_t gnpde_plan_workspace_bytes(int64_t R) {
  return 6 * align_up(sizeof(int32_t) * (size_t)(R + 1)) + align_up(cub_scan_bytes(R + 1)) + 256;
}

int gnpde_plan_build(const int32_t* rowptr, int64_t R, int32_t chunk, int32_t* items, int64_t items_capacity,
                     int32_t* heavy, int64_t heavy_capacity, int64_t* n_items, int64_t* n_heavy, int64_t* n_slots,
                     void* workspace, size_t workspace_bytes, void* stream) {
  GNPDE_REQUIRE(rowptr && items && n_items && n_heavy && n_slots && workspace, GNPDE_EINVAL,
                "plan_build: NULL pointer");
  GNPDE_REQUIRE(R >= 1 && chunk >= 1, GNPDE_EINVAL, "plan_build: bad R/chunk");
  GNPDE_REQUIRE(workspace_bytes >= gnpde_plan_workspace_bytes(R), GNPDE_EINVAL, "plan_build: workspace too small");
  hipStream_t s = as_stream(stream);
  char* ws = static_cast<char*>(workspace);
  const size_t a = align_up(sizeof(int32_t) * (size_t)(R + 1));
  int32_t* n_it = reinterpret_cast<int32_t*>(ws + 0 * a);
  int32_t* n_sl = reinterpret_cast<int32_t*>(ws + 1 * a);
  int32_t* n_hv = reinterpret_cast<int32_t*>(ws + 2 * a);
  int32_t* o_it = reinterpret_cast<int32_t*>(ws + 3 * a);
  int32_t* o_sl = reinterpret_cast<int32_t*>(ws + 4 * a);
  int32_t* o_hv = reinterpret_cast<int32_t*>(ws + 5 * a);
  void* tmp = ws + 6 * a;
  size_t tmp_bytes = workspace_bytes - 6 * a;
  // a zero count at index R makes the exclusive scan's last entry the total
  GNPDE_HIP(hipMemsetAsync(n_it + R, 0, sizeof(int32_t), s));
  GNPDE_HIP(hipMemsetAsync(n_sl + R, 0, sizeof(int32_t), s));
  GNPDE_HIP(hipMemsetAsync(n_hv + R, 0, sizeof(int32_t), s));
  plan_count_kernel<<<grid_for(R), 256, 0, s>>>(rowptr, R, chunk, n_it, n_sl, n_hv);
  GNPDE_LAUNCH_CHECK();
  GNPDE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, n_it, o_it, (int)(R + 1), s));
  GNPDE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, n_sl, o_sl, (int)(R + 1), s));
  GNPDE_HIP(hipcub::DeviceScan::ExclusiveSum(tmp, tmp_bytes, n_hv, o_hv, (int)(R + 1), s));
  int32_t tot[3] = {0, 0, 0};
  GNPDE_HIP(hipMemcpyAsync(&tot[0], o_it + R, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  GNPDE_HIP(hipMemcpyAsync(&tot[1], o_sl + R, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  GNPDE_HIP(hipMemcpyAsync(&tot[2], o_hv + R, sizeof(int32_t), hipMemcpyDeviceToHost, s));
  GNPDE_HIP(hipStreamSynchronize(s));
  *n_items = tot[0];
  *n_slots = tot[1];
  *n_heavy = tot[2];
  GNPDE_REQUIRE(tot[0] <= items_capacity, GNPDE_EINVAL, "plan_build: items capacity %lld < %d",
                (long long)items_capacity, tot[0]);
  GNPDE_REQUIRE(tot[2] <= heavy_capacity, GNPDE_EINVAL, "plan_build: heavy capacity %lld < %d",
                (long long)heavy_capacity, tot[2]);
  GNPDE_REQUIRE(tot[2] == 0 || heavy != nullptr, GNPDE_EINVAL, "plan_build: heavy is NULL");
  plan_emit_kernel<<<grid_for(R), 256, 0, s>>>(rowptr, R, o_it, o_sl, o_hv, n_it, reinterpret_cast<int4*>(items),
                                               reinterpret_cast<int4*>(heavy));
  GNPDE_LAUNCH_CHECK();
  return GNPDE_OK;
}

}  // extern "C"
