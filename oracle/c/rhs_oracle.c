/*
 * rhs_oracle.c — C restatement of the Laplacian ODE right-hand side.
 * TEST INFRASTRUCTURE ONLY: used by tests/ and by bench.py's cpu_baseline leg
 * (the timed CPU baseline on the GPU box's host cores).  Never linked into or
 * called by the product path.
 *
 * Restates (alimt1992/graph-neural-pde @ 2025-01-17):
 *   src/function_laplacian_diffusion.py:39-58  sparse_multiply: ax[b,i,:] =
 *       sum_{e: edge[b,0,e]=i} w[b,e] * x[b, edge[b,1,e], :]  (duplicates summed)
 *   src/function_laplacian_diffusion.py:69-77  f = alpha*(ax - x) [+ beta*x0],
 *       alpha = sigmoid(alpha_train) unless no_alpha_sigmoid
 * in float32 storage and float32 arithmetic (the reference's fp32 runs), over
 * a CSR built once per graph, OpenMP-parallel over rows.  Checked against the
 * numpy oracle (and through it the golden vectors) by tests/test_oracle_c.py.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* COO edge_index [B,2,E] (int64) -> block-diagonal CSR over R = B*N rows
 * (stable counting sort: in-row order = COO order).  w_coo [B*E] -> w_csr. */
int gnpde_oracle_csr(const int64_t* ei, int64_t B, int64_t E, int64_t N, const float* w_coo, int64_t* rowptr,
                     int32_t* col, float* w_csr) {
  const int64_t R = B * N, nnz = B * E;
  memset(rowptr, 0, sizeof(int64_t) * (size_t)(R + 1));
  for (int64_t b = 0; b < B; ++b)
    for (int64_t e = 0; e < E; ++e) {
      const int64_t s = ei[(b * 2 + 0) * E + e], d = ei[(b * 2 + 1) * E + e];
      if (s < 0 || s >= N || d < 0 || d >= N) return -1;
      rowptr[b * N + s + 1]++;
    }
  for (int64_t r = 0; r < R; ++r) rowptr[r + 1] += rowptr[r];
  int64_t* fill = (int64_t*)malloc(sizeof(int64_t) * (size_t)(R > 0 ? R : 1));
  if (!fill) return -2;
  memcpy(fill, rowptr, sizeof(int64_t) * (size_t)R);
  for (int64_t b = 0; b < B; ++b)
    for (int64_t e = 0; e < E; ++e) {
      const int64_t r = b * N + ei[(b * 2 + 0) * E + e];
      const int64_t p = fill[r]++;
      col[p] = (int32_t)(b * N + ei[(b * 2 + 1) * E + e]);
      w_csr[p] = w_coo[b * E + e];
    }
  free(fill);
  (void)nnz;
  return 0;
}

/* f[r,:] = a*(sum_p w[p] x[col[p],:] - x[r,:]) [+ beta*x0[r,:]] */
int gnpde_oracle_laplacian_rhs(const int64_t* rowptr, const int32_t* col, const float* w, int64_t R, int64_t C,
                               const float* x, const float* x0, float alpha_train, float beta_train,
                               int no_alpha_sigmoid, int add_source, float* f, int nthreads) {
  const float a = no_alpha_sigmoid ? alpha_train : 1.0f / (1.0f + expf(-alpha_train));
#ifdef _OPENMP
  if (nthreads > 0) omp_set_num_threads(nthreads);
#else
  (void)nthreads;
#endif
#pragma omp parallel for schedule(dynamic, 256)
  for (int64_t r = 0; r < R; ++r) {
    float* fr = f + r * C;
    for (int64_t c = 0; c < C; ++c) fr[c] = 0.0f;
    for (int64_t p = rowptr[r]; p < rowptr[r + 1]; ++p) {
      const float wp = w[p];
      const float* xr = x + (int64_t)col[p] * C;
      for (int64_t c = 0; c < C; ++c) fr[c] += wp * xr[c];
    }
    const float* xs = x + r * C;
    for (int64_t c = 0; c < C; ++c) {
      float v = a * (fr[c] - xs[c]);
      if (add_source) v += beta_train * x0[r * C + c];
      fr[c] = v;
    }
  }
  return 0;
}

int gnpde_oracle_max_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
