/*
 * gnpde.h — C ABI of the MI355X-native GRAND/BLEND ODE right-hand side.
 *
 * One shared library, libgnpde.so (graph-neural-pde_amd/gnpde/), built with
 * `hipcc --offload-arch=gfx950`.  Plain pointers and sizes only; no torch
 * types.  Every device pointer is owned by the caller (the Python host passes
 * torch tensors' data_ptr()); the library never allocates device memory and
 * keeps no state besides its kernels.  Every call enqueues on the caller's
 * `stream` (a hipStream_t passed as void*; NULL = legacy default stream) and
 * never synchronises, except gnpde_plan_build, which is documented as a
 * once-per-graph synchronous call.  All calls are graph-capturable except
 * gnpde_plan_build.
 *
 * Return codes: 0 ok, GNPDE_EINVAL (-1) invalid argument, GNPDE_EHIP (-2) HIP
 * runtime error, GNPDE_EUNSUPPORTED (-3) unsupported shape/dtype.  The message
 * of the last failure on the calling thread is returned by gnpde_last_error().
 *
 * Reference interfaces replaced (alimt1992/graph-neural-pde @ 2025-01-17):
 *   - the per-RHS COO->dense->matmul of LaplacianODEFunc.sparse_multiply,
 *     src/function_laplacian_diffusion.py:39-58, and of
 *     ODEFuncTransformerAtt.multiply_attention, src/function_transformer_attention.py:33-41;
 *   - the RHS epilogue f = sigma(alpha)(ax - x) [+ beta x0],
 *     src/function_laplacian_diffusion.py:69-77, src/function_transformer_attention.py:52-59;
 *   - SpGraphTransAttentionLayer.forward's Q/K projections, gathers, scaled_dot
 *     score and edge softmax, src/function_transformer_attention.py:224-266 and
 *     utils.softmax, src/utils.py:116-127;
 *   - the torchdiffeq stage combinations y0 + dt*sum(b_j k_j) the solver does
 *     between RHS calls (src/block_constant.py:46-51 calls odeint).
 *
 * Layout: graphs are block-diagonal over the batch: global node id
 * r = b*N + n (b < B, n < N), R = B*N rows.  Node features are row-major
 * [R, C] with leading dimension ld (elements).  A "CSR" here is rowptr[R+1],
 * col[nnz] (global node ids), perm[nnz] (CSR position -> COO edge id b*E+e).
 * Grouping by source (edge_index[:,0]) gives the aggregation CSR; grouping by
 * destination (edge_index[:,1]) gives the CSC used for destination-grouped
 * softmax (attention_norm_idx = 1).
 */
#ifndef GNPDE_H_
#define GNPDE_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define GNPDE_ABI_VERSION 8

#define GNPDE_OK 0
#define GNPDE_EINVAL (-1)
#define GNPDE_EHIP (-2)
#define GNPDE_EUNSUPPORTED (-3)

/* flags for the RHS epilogue */
#define GNPDE_EPI_PLAIN 0          /* f = ax                                   */
#define GNPDE_EPI_RHS 1            /* f = a*(ax - x) [+ b*x0]                  */
#define GNPDE_ALPHA_SIGMOID 2      /* a = sigmoid(*alpha) instead of *alpha    */
#define GNPDE_ADD_SOURCE 4         /* add b*x0 (b = *beta)                      */

/* score modes of the attention RHS (function_transformer_attention.py:246-259) */
#define GNPDE_SCORE_REFERENCE 0    /* fork scaled_dot: q_src . (sum_e' k_dst(e')) / sqrt(dk)      */
#define GNPDE_SCORE_DOT 1          /* per-edge scaled_dot: q_src . k_dst / sqrt(dk) (upstream)    */
#define GNPDE_SCORE_EXP_KERNEL 2   /* ov^2 exp(-|q_src - k_dst|^2 / (2 ls^2))                     */
#define GNPDE_SCORE_COSINE 3       /* cosine similarity, eps 1e-5                                 */
#define GNPDE_SCORE_PEARSON 4      /* centred cosine similarity                                   */
#define GNPDE_SCORE_UNIFORM 5      /* every score 0: the fork's scaled_dot under source-grouped    */
                                   /* softmax (norm_idx 0), where all scores of a group are equal  */

int gnpde_abi_version(void);
const char* gnpde_last_error(void);
/* Hash of the sources the library was built from (graph-neural-pde_amd/srchash.py). */
const char* gnpde_build_id(void);

/* ---------------------------------------------------------------- graph build
 * COO edge_index [B,2,E] (int64, values in [0,N) — caller-validated) -> CSR
 * grouped by row `key_row` (0 = source, 1 = destination).  Stable: inside a
 * row, edges keep their COO order.  Replaces the per-call index building of
 * function_laplacian_diffusion.py:41-44 (done once per graph here).         */
size_t gnpde_csr_workspace_bytes(int64_t B, int64_t E, int64_t N);
int gnpde_csr_build(const int64_t* edge_index, int64_t B, int64_t E, int64_t N, int key_row,
                    int32_t* rowptr, int32_t* col, int32_t* perm,
                    void* workspace, size_t workspace_bytes, void* stream);

/* rowidx[p] = the row of CSR position p (once per graph; drives the
 * edge-parallel attention-weight kernels).                                   */
int gnpde_csr_rowidx(const int32_t* rowptr, int64_t R, int64_t nnz, int32_t* rowidx, void* stream);

/* w_out[p] = mean_{h<H} w_in[perm[p]*H + h]  (H = 1: plain permutation).
 * Head-mean of attention weights, function_laplacian_diffusion.py:45-49.    */
int gnpde_gather_weights_f32(const float* w_in, int64_t nnz, int H, const int32_t* perm, float* w_out,
                             void* stream);

/* ---------------------------------------------------------------- block weight producers
 * out[i] = mean_{h<H} att[i*H + h]  (H = 1: copy), and when gamma != NULL
 * out[i] = mean * (1 - sigmoid(*gamma)) + ew[i] * sigmoid(*gamma)  (COO order,
 * n = B*E).  gamma is a device scalar (pre-sigmoid).  Replaces
 * MixedODEblock.get_mixed_attention, src/block_mixed.py:29-33, and the
 * head mean of HardAttODEblock.forward, src/block_transformer_hard_attention.py:42,60. */
int gnpde_mix_weights_f32(const float* att, int H, const float* ew, const float* gamma, int64_t n, float* out,
                          void* stream);

/* w_out[e] = w_in[e] / (sum of w_in over e's group + 1e-16), groups = the rows
 * of a grouped CSR (rowptr[R+1], perm[nnz] = CSR position -> COO edge id),
 * COO order in and out; fixed summation order (deterministic).  Replaces
 * HardAttODEblock.renormalise_attention, src/block_transformer_hard_attention.py:32-35.
 * ABI 7: a workspace of gnpde_group_normalize_workspace_bytes(nnz) (the weights in
 * group order, so each group's sum streams a contiguous run). */
size_t gnpde_group_normalize_workspace_bytes(int64_t nnz);
int gnpde_group_normalize_f32(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, const float* w_in,
                              float* w_out, void* workspace, size_t workspace_bytes, void* stream);

/* *out = torch.quantile(v[0:n], q) (linear interpolation; rank q*(n-1) in
 * fp32, ATen's lerp) written to DEVICE memory; radix sort into the workspace.
 * The attention-sampling threshold of src/block_transformer_hard_attention.py:52. */
size_t gnpde_quantile_workspace_bytes(int64_t n);
int gnpde_quantile_f32(const float* v, int64_t n, double q, float* out, void* workspace, size_t workspace_bytes,
                       void* stream);

/* The training-mode attention sampling as a weight mask over the full edge list
 * (src/block_transformer_hard_attention.py:52-55): out[i] = v[i] > *thr ? v[i] : 0,
 * *count (device int64) = the retained edges.  With these weights the RHS over the
 * full graph equals the RHS over the compacted edge list (zero weights add exact
 * zeros), so a training forward needs no new CSR / plan.  thr: device (the
 * gnpde_quantile_f32 output).                                                 */
int gnpde_threshold_mask_f32(const float* v, int64_t n, const float* thr, float* out, int64_t* count, void* stream);
/* The sampled graph of HardAttODEblock training over a work plan (ABI 7;
 * src/block_transformer_hard_attention.py:52-56 keeps the edges above the
 * threshold and integrates over that edge list): for every plan item
 * {row, edge_begin, edge_end, slot} of gnpde_plan_build, the positions of
 * [edge_begin, edge_end) whose weight w (grouped order, e.g. gnpde_threshold_mask_f32
 * then gnpde_gather_weights_f32) is nonzero are written, in order, to
 * col_out / w_out from edge_begin on, and items_out = {row, edge_begin,
 * edge_begin + kept, slot}.  Launching K1 with items_out / col_out / w_out (and the
 * plan's heavy entries unchanged) aggregates the retained edges only, in the
 * order and hub chunks of the full plan: the same result as the masked full graph.
 * No host synchronisation; outputs the size of the inputs; no aliasing.        */
int gnpde_compact_items_f32(const int32_t* items, int64_t n_items, const int32_t* col, const float* w,
                            int32_t* col_out, float* w_out, int32_t* items_out, void* stream);

/* deg[r] = #{p : idx[p] == r}, r < R (memset + integer atomics: deterministic).
 * With idx = the aggregation CSR's col this is the in-degree used by the
 * reference-mode key sum.                                                   */
int gnpde_indegree_i32(const int32_t* idx, int64_t nnz, int64_t R, int32_t* deg, void* stream);

/* ---------------------------------------------------------------- graph normalisation
 * ODEblock.reset_graph_data (src/base_classes.py:70-90) with the intended
 * semantics of add_remaining_self_loops / get_rw_adj / gcn_norm_fill_val
 * (src/utils.py:16-42, :215-233, :177-194; pinned by test/test_utils.py:111-161
 * and test/test_function_laplacian_diffusion.py:56-86), once per graph.
 *
 * gnpde_self_loops_count: nonloop[b] = #{e : edge_index[b,0,e] != edge_index[b,1,e]}
 *   written to HOST memory (SYNCHRONOUS, like gnpde_plan_build).
 * gnpde_add_self_loops: per batch element, the K non-loop edges in COO order,
 *   then one loop (n, n) per node n < N whose weight is the weight of the node's
 *   LAST existing loop in COO order, or `fill` (w NULL: every weight 1).  K must
 *   be the same for every batch element (the [B,2,K+N] layout); outputs
 *   ei_out [B,2,K+N] int64, w_out [B,K+N] fp32.
 * gnpde_norm_weights_f32: fac[r] = deg(r)^-1 (RW_*) or deg^-1/2 with inf -> 0
 *   (GCN), deg summed sequentially in COO order over the grouped CSR (rowptr,
 *   perm) of gnpde_csr_build — grouped by source (key_row 0) for RW_ROW, by
 *   destination (key_row 1) for RW_COL and GCN; then
 *   RW_ROW: w_out = fac[row] * w,  RW_COL: w_out = w * fac[col],
 *   GCN:    w_out = fac[row] * w * fac[col]  (fac [B*N] is caller scratch).  */
#define GNPDE_NORM_RW_ROW 0  /* get_rw_adj(norm_dim=0)        */
#define GNPDE_NORM_RW_COL 1  /* get_rw_adj(norm_dim=1)        */
#define GNPDE_NORM_GCN 2     /* gcn_norm_fill_val             */
size_t gnpde_self_loops_workspace_bytes(int64_t B, int64_t E, int64_t N);
int gnpde_self_loops_count(const int64_t* edge_index, int64_t B, int64_t E, int64_t* nonloop, void* workspace,
                           size_t workspace_bytes, void* stream);
int gnpde_add_self_loops(const int64_t* edge_index, const float* w, int64_t B, int64_t E, int64_t N, float fill,
                         int64_t K, int64_t* ei_out, float* w_out, void* workspace, size_t workspace_bytes,
                         void* stream);
int gnpde_norm_weights_f32(const int64_t* edge_index, const float* w, int64_t B, int64_t E, int64_t N,
                           const int32_t* rowptr, const int32_t* perm, int mode, float* fac, float* w_out,
                           void* stream);

/* ---------------------------------------------------------------- work plan
 * Splits rows with more than `chunk` edges into balanced chunks so that one
 * power-law hub does not serialise a wavefront.  items[n_items] is int4
 * {row, edge_begin, edge_end, slot} (slot = -1: the item owns its row;
 * slot >= 0: partial-sum slot); heavy[n_heavy] is int4 {row, first_slot,
 * n_chunks, 0}.  Capacity: items >= R + 2*nnz/chunk + 1, heavy >= nnz/chunk + 1.
 * SYNCHRONOUS (copies the two counts to the host); call once per graph.     */
int gnpde_plan_build(const int32_t* rowptr, int64_t R, int32_t chunk,
                     int32_t* items, int64_t items_capacity, int32_t* heavy, int64_t heavy_capacity,
                     int64_t* n_items, int64_t* n_heavy, int64_t* n_slots,
                     void* workspace, size_t workspace_bytes, void* stream);
size_t gnpde_plan_workspace_bytes(int64_t R);

/* ---------------------------------------------------------------- fused solver epilogue
 * Optional stage outputs of the RHS kernels, so a Runge-Kutta stage combination
 * y0 + dt*sum_j b_j k_j is produced by the same pass that computes k_i (no
 * separate read of k_i, no extra launch).  A stage has nk shared operand
 * arrays k[0..nk-1] (each read once per row however many outputs use it); with
 * f = the RHS value of row r:
 *   f_out[r]    = f                                            (f_out may be NULL)
 *   o[i].out[r] = cb*base[r] + cf*f + sum_{j<nk} o[i].c[j]*k[j][r]   for i < n_out
 * base may be NULL (0), equal to the RHS input x (the row already read by the
 * epilogue is reused) or equal to o[i].out (in-place accumulation).  Every
 * array has the leading dimension ldf of the RHS output.  No output may alias
 * the RHS input x (other rows of x are still being gathered).
 * out_rows (NULL = identity): the o[i].out stores of row r go to row
 * out_rows[r] instead (base, k and f_out stay at row r) — the last step of a
 * solve run in a renumbered node order writes its result straight into the
 * caller's numbering (gnpde.integrator); it must be a permutation of [0, R).
 * dot_rows (NULL = none; fp32 state, power-of-two lanes per row): per row,
 *   dot_rows[r] (+)= dot_coef * sum_c f[r,c] * dot_with[r,c]   (fp64; "+=" when
 * dot_accumulate), summed over the row's lanes in a fixed order — the per-row
 * terms of a parameter gradient <f, y> that the caller reduces once
 * (gnpde_sum_f64), instead of a separate pass re-reading f.
 * err_rows (NULL = none): the error estimate of an embedded Runge-Kutta pair
 * (torchdiffeq's RKAdaptiveStepsizeODESolver: error_ratio = RMS(e / tol)):
 *   e      = err.cb*err.base + err.cf*f + sum_{j<nk} err.c[j]*k[j]   (err.out unused)
 *   y1     = the RHS input x (err_y1 = -1), err_y0 itself (err_y1 = -2, ABI 8: tol =
 *            atol + rtol |y0|, the scale of torchdiffeq's initial-step selection) or
 *            the value of output err_y1
 *   tol    = atol + rtol * max(|err_y0|, |y1|)
 *   err_rows[r] = sum_c (e / tol)^2     (fp64, the row's lanes in a fixed order)
 * which the caller sums (gnpde_sum_f64) into the squared norm of one step.
 * scale_rows (NULL = none; ABI 8; with err_rows, the plain-weight K1 only, not beside
 * dot_rows): scale_rows[r] = sum_c (err_y0 / tol)^2 — with e = f and err_y1 = -2 the
 * f0 launch of an adaptive solve yields both squared sums of the initial-step
 * selection (gnpde_initial_step_rows).
 * coef_scale (NULL = 1): a device fp32 scalar multiplying every cf and c[j] of the
 * outputs and of err (not cb): the step size of an adaptive solve, so the
 * launches of a step do not change with it (hipGraph-replayable, one graph per
 * step whatever dt).
 * f_lin (0 = off): the RHS value becomes f = x + coef_scale*f_lin*f before any
 * store or combination (x = the RHS input row): for an affine RHS f(y) = L y + s
 * evaluated on the input k WITHOUT the source term (flags: no GNPDE_ADD_SOURCE),
 * f(y0 + h k) = k + h L k with k = f(y0) — an adaptive step's first stage derivative
 * without materialising its stage input y0 + h k (gnpde.integrator, ABI 5).
 * unscaled_outs (0 = none; ABI 6): bit i set — output i takes its cf and c[j]
 * WITHOUT coef_scale (the error term always takes it): a combination whose
 * operands already carry the step size, e.g. the next step's f0 = sum_p B[p] u_p
 * of the affine Krylov step (u_p = (h L)^p f0, gnpde.integrator).
 * A k operand (or base) equal to the RHS input x reuses the row already read.
 * err_rows and 3..6 operands take the wide epilogue (operands loaded after the
 * aggregation); since ABI 7 it carries dot_rows too, beside err_rows or with up to
 * 6 operands (a second fp64 row sum: the adaptive adjoint's alpha integrand
 * <L^T a_i, y_i> in the launch that forms the next adjoint stage input and its
 * error rows, gnpde.integrator), fused into the plain-weight
 * K1 (gnpde_spmm_rhs_f32 / _bf16); the attention kernels return
 * GNPDE_EUNSUPPORTED for it (the caller applies it with gnpde_stage_apply_*).
 * dense_out (NULL = none; ABI 8; plain-weight K1 with err_rows only): the dense
 * output of the adaptive step folded into its last launch.  With the device
 * fp64 scalars t0 = dense_t[0] (the step's start), t_out = dense_t[1] and
 * h = *dense_dt (the step size), when t0 < t_out <= t0 + h (the step crosses the
 * output time; wave-uniform, nothing is written otherwise):
 *   x = (t_out - t0)/h, the basis w = {cy0 + cy1 + cym, h cy1, h cym, cf0, cf1}
 *   of torchdiffeq's 4th-order interpolant (cy0 = 1 - 11x^2 + 18x^3 - 8x^4,
 *   cy1 = -5x^2 + 14x^3 - 8x^4, cym = 16x^2 - 32x^3 + 16x^4,
 *   cf0 = h (x - 4x^2 + 5x^3 - 2x^4), cf1 = h (x^2 - 3x^3 + 2x^4)),
 *   out[dense_rows[r]] = sum_m w[m] (dense_m[m][0] o[0].base[r]
 *                        + sum_{j<nk} dense_m[m][1+j] k[j][r] + dense_m[m][7] f[r])
 * (coefficients formed in fp64, applied in fp32; f after f_lin), out = *dense_out
 * (a device slot holding the output array: the launch can be captured once and
 * its output redirected per solve).  dense_tab: device scratch of
 * GNPDE_STAGE_MAX_K + 3 floats holding the crossing flag and the coefficients of
 * the launch's step, which an EARLIER launch of the same step forms: a K1 launch
 * whose stage sets dense_tab, dense_t, dense_dt and dense_m but not dense_out writes
 * them (a one-wavefront launch ahead of its aggregation) — the first launch of
 * the step, so the one that applies them reads them into scalar registers.    */
#define GNPDE_STAGE_MAX_OUT 2
#define GNPDE_STAGE_MAX_K 6
#define GNPDE_DENSE_BASIS 5
typedef struct {
  float* out;
  const float* base;
  float cb;
  float cf;
  float c[GNPDE_STAGE_MAX_K];
} gnpde_stage_out_t;

typedef struct {
  float* f_out;
  int n_out;
  gnpde_stage_out_t o[GNPDE_STAGE_MAX_OUT];
  int nk;
  const float* k[GNPDE_STAGE_MAX_K];
  const int32_t* out_rows;
  const float* dot_with;
  double* dot_rows;
  double dot_coef;
  int dot_accumulate;
  double* err_rows;
  gnpde_stage_out_t err;
  const float* err_y0;
  int err_y1;
  double atol;
  double rtol;
  const float* coef_scale;
  float f_lin;
  int unscaled_outs;
  float* const* dense_out;
  const int32_t* dense_rows;
  const double* dense_t;
  const double* dense_dt;
  float* dense_tab;
  float dense_m[GNPDE_DENSE_BASIS][GNPDE_STAGE_MAX_K + 2];
  double* scale_rows;
} gnpde_stage_epilogue_t;

/* The stage epilogue as a pass of its own, over rows [0, R) of C columns
 * (leading dimension ld, every array of the stage included): f [R, ld] is the
 * RHS value (NULL: every cf term is 0 — a plain combination such as a stage
 * input y0 + dt*b0*k0 or dense output), x the RHS input (needed when a base is
 * x or err_y1 = -1; may be NULL otherwise).  Same arithmetic, per element, as
 * the fused epilogue (fp32; err_rows in fp64).  bf16: every row array is bf16
 * (the struct's float* reinterpreted), the arithmetic fp32.  Used by the
 * adaptive solvers for the attention RHS kernels that fuse only the fixed-grid
 * stages, and for the pre-step and dense-output combinations.               */
int gnpde_stage_apply_f32(int64_t R, int64_t C, int64_t ld, const float* f, const float* x,
                          const gnpde_stage_epilogue_t* stage, void* stream);
int gnpde_stage_apply_bf16(int64_t R, int64_t C, int64_t ld, const uint16_t* f, const uint16_t* x,
                           const gnpde_stage_epilogue_t* stage, void* stream);

/* ---------------------------------------------------------------- K1: SpMM RHS
 * ax[r,:] = sum_{p in row r} w[p] * x[col[p],:]
 * f[r,:]  = ax                                  (flags & 1 == 0)
 *         = a*(ax - x[r,:]) [+ b*x0[r,:]]        (GNPDE_EPI_RHS)
 * a = *alpha or sigmoid(*alpha), b = *beta: device scalars (no host sync).
 * partials: n_slots*C floats of scratch (NULL if n_slots == 0; n_slots from
 * gnpde_plan_build); n_slots*C*4 must stay below 0xffffff00 bytes (the hub
 * partials are addressed with 32-bit buffer offsets): GNPDE_EUNSUPPORTED past
 * it — plan the graph with a larger chunk.
 * heavy: the hub table of gnpde_plan_build.  The chunks of a hub row are
 * combined inside the launch by the chunk that finishes last, which it learns
 * from an arrival ticket kept in the 4th word of the row's heavy entry
 * (plan_build writes 0; every launch leaves 0).  Launches that share one plan
 * must therefore be ordered (one stream, or events) — never concurrent.
 * stage: NULL -> f[r,:] is stored to f; otherwise the stage epilogue above
 * decides what is stored (f is ignored).
 * Replaces function_laplacian_diffusion.py:39-77 per RHS evaluation.        */
int gnpde_spmm_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                       const int32_t* col, const float* w, int64_t C,
                       const float* x, int64_t ldx, const float* x0, int64_t ldx0,
                       const float* alpha, const float* beta, int flags,
                       float* f, int64_t ldf, float* partials, int64_t n_slots,
                       const gnpde_stage_epilogue_t* stage, void* stream);

/* K1 on bfloat16 storage (configs[3], BLEND in bf16): x, x0, f and every
 * stage pointer of `stage` address bf16 arrays (raw uint16 bits; the stage
 * struct's float* fields are reinterpreted); weights, alpha, beta and the
 * partials stay fp32, and every sum and the epilogue run in fp32 — only the
 * stored rows are rounded (nearest even).  Otherwise as gnpde_spmm_rhs_f32.  */
int gnpde_spmm_rhs_bf16(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                        const int32_t* col, const float* w, int64_t C, const uint16_t* x, int64_t ldx,
                        const uint16_t* x0, int64_t ldx0, const float* alpha, const float* beta, int flags, uint16_t* f,
                        int64_t ldf, float* partials, int64_t n_slots, const gnpde_stage_epilogue_t* stage,
                        void* stream);

/* K1 with the attention weights computed on the fly for the fork's scaled_dot
 * (reference score mode) under destination-grouped softmax (attention_norm_idx
 * 1): w_p = mean_h exp(cs[row,h] - m[col_p,h]) * rl[col_p,h], cs [R,H] fp64 node
 * scores (gnpde_ref_scores_f32), m [R,H] fp64 / rl [R,H] group statistics
 * (gnpde_softmax_stats_f32 / gnpde_seg_softmax_f32 over the CSC), or, when
 * mr is given (heads == 2, 16-byte aligned), the packed statistics records
 * those kernels write into mr (GNPDE_STATS_RECORD_FLOATS(heads) floats per
 * group: m[0..h-1], then rl[0..h-1]): one 16-byte load per edge.  Every
 * statistics kernel stores the group max rounded to fp32 (exact in both forms)
 * and the sum relative to it, so both forms hold the same values.
 * Equals gnpde_attn_weights_f32 + gnpde_spmm_rhs_f32 bit for bit, in one pass:
 * ODEFuncTransformerAtt.forward, function_transformer_attention.py:44-59.
 * Other arguments as gnpde_spmm_rhs_f32.                                     */
#define GNPDE_STATS_RECORD_FLOATS(h) ((2 * (h) + 3) & ~3)
int gnpde_attn_ref_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                           const int32_t* col, const double* cs, const double* m, const float* rl, const float* mr,
                           int64_t heads,
                           int64_t C, const float* x, int64_t ldx, const float* x0, int64_t ldx0, const float* alpha,
                           const float* beta, int flags, float* f, int64_t ldf, float* partials, int64_t n_slots,
                           const gnpde_stage_epilogue_t* stage, void* stream);

/* The per-edge scaled_dot attention RHS under source-grouped softmax
 * (attention_norm_idx 0; upstream GRAND's transformer RHS) in ONE aggregation
 * pass over the CSR plan (csrc/flash.hip): every row slot scores the edges it
 * gathers, s_e,h = q[row,h] . k[col_e,h] / sqrt(dk), forms its group's
 * statistics (max M_h, sum L_h of exp(s - M_h)) and aggregates with
 *   w_e = (1/H) sum_h exp(s_e,h - M_h) / (L_h + 1e-16)
 * = multiply_attention with the head mean of utils.softmax over edge_index[0]
 * (function_transformer_attention.py:33-41, 246-266; src/utils.py:116-127),
 * then the RHS epilogue, or a single-output stage epilogue without a dot
 * term (the forward integrator's; others: GNPDE_EUNSUPPORTED), as
 * gnpde_spmm_rhs_f32.  Replaces
 * gnpde_seg_softmax_f32(out_kind 0) + gnpde_spmm_rhs_f32 (no [nnz] weights).
 * q, k: [R, ldqk] fp32 (gnpde_linear_f32), 16-byte aligned rows.  Hub rows
 * (heavy entries of the plan): each chunk keeps its own statistics and
 * per-head sums in a partial slot, merged in-launch by the last chunk to
 * arrive (heavy[].w tickets, as K1).  workspace:
 * gnpde_attn_dot_workspace_floats(heads, C, n_slots) floats, 16-byte aligned.
 * Shapes:
 * gnpde_attn_dot_supported(heads, dk, C) != 0 (heads in {1, 2, 4}, dk % 4 ==
 * 0, heads*dk in {8, 16, 32, 64}, C % 4 == 0, C <= 256); otherwise
 * GNPDE_EUNSUPPORTED.  Exponentials in base 2 (1-2 ulp from expf).
 * dst_stats != NULL: destination-grouped softmax (attention_norm_idx 1)
 * instead — the packed statistics records of every destination
 * (GNPDE_STATS_RECORD_FLOATS(heads) floats: m[h] then rl[h], from
 * gnpde_seg_softmax_f32 over the CSC, 16-byte aligned) weight each scored
 * edge, w_e = (1/H) sum_h exp(s_e,h - m[c,h]) rl[c,h]: replaces
 * gnpde_attn_weights_f32 + gnpde_spmm_rhs_f32.                              */
int gnpde_attn_dot_supported(int64_t heads, int64_t dk, int64_t C);
int64_t gnpde_attn_dot_workspace_floats(int64_t heads, int64_t C, int64_t n_slots);
int gnpde_attn_dot_rhs_f32(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                           const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads, int64_t dk,
                           const float* dst_stats, int64_t C, const float* x, int64_t ldx, const float* x0, int64_t ldx0,
                           const float* alpha, const float* beta, int flags, float* f, int64_t ldf, float* workspace,
                           int64_t n_slots, const gnpde_stage_epilogue_t* stage, void* stream);
/* The same over a bf16 state (x, x0, f and the stage rows bf16, 8-byte aligned
 * 4-element slices; q, k, dst_stats and the workspace fp32): source-grouped
 * softmax (dst_stats NULL) with the plain RHS or a single-output stage only,
 * GNPDE_EUNSUPPORTED otherwise (the binding then takes K2 + gnpde_spmm_rhs_bf16). */
int gnpde_attn_dot_rhs_bf16(const int32_t* items, int64_t n_items, int32_t* heavy, int64_t n_heavy,
                            const int32_t* col, const float* q, const float* k, int64_t ldqk, int64_t heads,
                            int64_t dk, const float* dst_stats, int64_t C, const void* x, int64_t ldx, const void* x0,
                            int64_t ldx0, const float* alpha, const float* beta, int flags, void* f, int64_t ldf,
                            float* workspace, int64_t n_slots, const gnpde_stage_epilogue_t* stage, void* stream);

/* ---------------------------------------------------------------- attention
 * Node-level projection on the matrix cores (K % 16 == 0, K <= 128: exact
 * three-piece bf16 splits of both operands on v_mfma_f32_32x32x16_bf16, f32-GEMM
 * accuracy; other shapes: v_mfma_f32_32x32x2_f32):
 *   out[r, j] = sum_k x[r,k] * W[j,k] + bias[j], j < Nout; columns [0, split)
 *   go to out_a (ld lda), [split, Nout) to out_b (ld ldb).
 * Replaces the nn.Linear Q/K of function_transformer_attention.py:224-225.  */
int gnpde_linear_f32(const float* x, int64_t R, int64_t K, int64_t ldx, const float* W, const float* bias,
                     int64_t Nout, int64_t split, float* out_a, int64_t lda, float* out_b, int64_t ldb,
                     void* stream);
/* The same projection of a bf16 state (x: [R, ldx] bf16): the elements are widened
 * to fp32 exactly on load, so the outputs equal gnpde_linear_f32 of the fp32 copy of
 * x bit for bit (a bf16 state's per-edge attention scores without that copy). */
int gnpde_linear_bf16(const void* x, int64_t R, int64_t K, int64_t ldx, const float* W, const float* bias,
                      int64_t Nout, int64_t split, float* out_a, int64_t lda, float* out_b, int64_t ldb,
                      void* stream);

/* Weight gradient of the projection: gW[m, k] = sum_r gy[r, m] * x[r, k]
 * (gy [R, M] ld ldg = dL/d[q | k], x [R, K] ld ldx; gW [M, K] ld ldw), the
 * backward of nn.Linear's weight for the Q / K of
 * function_transformer_attention.py:224-225.  fp32 matrix cores
 * (v_mfma_f32_32x32x2_f32), the rows split over up to 512 wavefronts (at least
 * 128 rows each, and no more partial tiles than 64 MiB hold) whose partial tiles
 * are summed in wave order (deterministic).  workspace:
 * gnpde_linear_wgrad_workspace_bytes(R, M, K) bytes.                         */
size_t gnpde_linear_wgrad_workspace_bytes(int64_t R, int64_t M, int64_t K);
int gnpde_linear_wgrad_f32(const float* gy, int64_t R, int64_t M, int64_t ldg, const float* x, int64_t K, int64_t ldx,
                           float* gW, int64_t ldw, void* workspace, size_t workspace_bytes, void* stream);

/* Reference-mode node scores (fork scaled_dot, function_transformer_attention.py:249):
 *   S_b = Wk * (sum_n indeg(n) x_n) + (sum_n indeg(n)) bk    (fp64)
 *   cs[r,h] = (q_r,h . S_b,h) / sqrt(dk),  q = Wq x + bq      (fp64 out)
 * indeg: in-degree per global node (int32, R); ws: gnpde_keysum_workspace_bytes
 * (scratch, no state between calls).  Three launches: indegree-weighted column
 * sums over ~256 fp64 row tiles; one workgroup per batch element summing the
 * tiles in fixed order and forming S_b, U = Wq^T S / sqrt(dk) and v; the node
 * scores cs = x U + v.  attention_dim <= 4096.                               */
size_t gnpde_keysum_workspace_bytes(int64_t B, int64_t N, int64_t C, int64_t att);
int gnpde_ref_scores_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                         const float* Wq, const float* bq, const float* Wk, const float* bk,
                         int64_t att, int64_t heads, double* cs, void* workspace, size_t workspace_bytes,
                         void* stream);

/* The same in two phases, for a state split into column stripes (gnpde.dist):
 * S and cs are linear in the columns, so each stripe forms its share and the
 * caller sums the shares over the stripes between the phases (one all-reduce of
 * S [B, att] fp64, one of cs [R, heads] fp64):
 *   gnpde_ref_keysum_f32:             S[b] = Wk xbar_b + (sum_n indeg(n)) bk   (fp64 [B][att];
 *                                     the stripe's columns of Wk, bk on one stripe only)
 *   gnpde_ref_scores_from_keysum_f32: cs[r,h] = q_r,h . S_b,h / sqrt(dk) from a given S
 *                                     (the stripe's columns of Wq, bq on one stripe only).
 * x, Wk, Wq: the stripe's columns (C of them, contiguous [att, C] weights);
 * workspace as gnpde_ref_scores_f32.                                          */
int gnpde_ref_keysum_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const int32_t* indeg,
                         const float* Wk, const float* bk, int64_t att, double* S, void* workspace,
                         size_t workspace_bytes, void* stream);
int gnpde_ref_scores_from_keysum_f32(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const double* S,
                                     const float* Wq, const float* bq, int64_t att, int64_t heads, double* cs,
                                     void* workspace, size_t workspace_bytes, void* stream);

/* Destination- or source-grouped softmax statistics over a grouped CSR
 * (items from gnpde_plan_build over the CSC for norm_idx=1, the CSR for
 * norm_idx=0; gidx = the OTHER endpoint of each edge):
 * m[g,h] = max_e s_e,h rounded to fp32 (stored as fp64), rl[g,h] = 1/(sum_e exp(s_e,h - m) + 1e-16).
 * partials: 2*heads doubles per plan slot.
 * Edge scores by `mode` from cs (REFERENCE) or q/k (per-edge modes).
 * Groups of 8 lanes per item: plan it with a small chunk (e.g. 64).
 * m, rl and mr (packed records, see gnpde_attn_ref_rhs_f32) are each optional;
 * m and rl come as a pair, and at least one of the two forms is written.
 * Restates utils.softmax, src/utils.py:116-127.                              */
int gnpde_softmax_stats_f32(const int32_t* items, int64_t n_items, const int32_t* heavy, int64_t n_heavy,
                            const int32_t* gidx, int group_is_dst, int mode, int64_t heads, int64_t dk,
                            const double* cs, const float* q, const float* k, int64_t ldqk,
                            float score_p0, float score_p1,
                            double* m, float* rl, float* mr, double* partials, void* stream);

/* Head-mean attention weights in aggregation-CSR order (edge-parallel):
 *   w[p] = (1/h) sum_h exp(s_p,h - m[g,h]) * rl[g,h],  g = src (norm_idx 0) or dst (1)
 * (utils.softmax then attention.mean(dim=2), function_transformer_attention.py:34).
 * The attention RHS is then gnpde_spmm_rhs_f32 with these weights
 * (multiply_attention :33-41 + forward :52-59).                              */
int gnpde_attn_weights_f32(const int32_t* rowidx, const int32_t* col, int64_t nnz, int norm_idx, int mode,
                           int64_t heads, int64_t dk, const double* cs, const float* q, const float* k, int64_t ldqk,
                           float score_p0, float score_p1, const double* m, const float* rl, float* w_out,
                           void* stream);

/* K2: edge-block segmented softmax over a grouped CSR (the aggregation CSR
 * for norm_idx 0, the CSC for norm_idx 1; gidx = the other endpoint, rowidx =
 * the group of every position, group_is_dst as in gnpde_softmax_stats_f32).
 * One wavefront per item = at most EB consecutive edges (EB =
 * gnpde_seg_block_edges(mode, heads, dk); 0 means unsupported): items are
 * int4 {e_begin, e_end, -1, first_group} covering consecutive whole groups
 * (packed greedily up to EB edges); chunk_items {e_begin, e_end, slot, group}
 * split groups of degree > EB, heavy {group, first_slot, n_chunks, 0} lists
 * those groups (partials: 2*heads doubles per slot; m/rl scratch).
 * Reference scores with out_kind 1 over the CSC (norm_idx 1) also take, at the
 * front of `items`, n_hub_items HUB CHUNK items {e_begin, e_end, slot, hub}
 * (gnpde_seg_long_edges()-edge chunks of the longer groups, one wavefront each;
 * heavy[hub] = {group, first_slot, n_chunks, 0} lists those groups, n_heavy of
 * them, and partials holds 2*heads doubles per slot: the last chunk of a group to
 * arrive merges its slots in chunk order and resets heavy[hub].w, so two launches
 * on one plan must not overlap) and then n_long_items LONG items {e_begin, e_end,
 * -2, group} (a whole group of at most gnpde_seg_long_edges() edges, one wavefront
 * each); the rest are whole-group items, taken two per wavefront, and
 * n_chunk_items is 0.  (n_hub_items = n_long_items = 0 for other plans.)
 * gnpde_seg_plan_build builds them from a HOST copy of rowptr into HOST
 * arrays (plain C++, once per graph; capacities: items >= R, chunk_items >=
 * nnz/eb + R, heavy >= nnz/eb + 1).  When chunk_items == items + 4*n_items
 * (stored back to back) both item kinds run in one launch.
 *   out_kind 0: w[p] = (1/H) sum_h softmax_p,h in grouped order (per-edge
 *               modes with norm_idx 0: the aggregation weights of K1);
 *   out_kind 1: m[g,h] = max (fp64), rl[g,h] = 1/(sum exp(s - m) + 1e-16),
 *               into m/rl and/or the packed records mr (gnpde_attn_ref_rhs_f32).
 * Per-group max and sum come from segmented scans across the lanes (fixed
 * order, deterministic).  Restates utils.softmax, src/utils.py:116-127, with
 * the scores of function_transformer_attention.py:246-259 and the head mean of
 * :34.  Returns GNPDE_EUNSUPPORTED for shapes outside the kernel (dk % 4 != 0,
 * non-power-of-two teams, uniform scores, reference scores with out_kind 0).  */
int gnpde_seg_block_edges(int mode, int64_t heads, int64_t dk);
/* Edges of one long item of the reference statistics (whole groups up to it,
 * chunks of it beyond): the plan builder's unit. */
int gnpde_seg_long_edges(void);
/* Edges one wavefront covers in ONE pass over a long item of `heads` heads
 * (<= gnpde_seg_long_edges()): the long-item size of a small graph's plan, whose
 * launch is latency-bound (every item one pass; longer groups as hub chunks). */
int gnpde_seg_long_pass_edges(int64_t heads);
int gnpde_seg_plan_build(const int32_t* rowptr, int64_t R, int32_t eb, int32_t* items, int64_t items_capacity,
                         int32_t* chunk_items, int64_t chunks_capacity, int32_t* heavy, int64_t heavy_capacity,
                         int64_t* n_items, int64_t* n_chunks, int64_t* n_heavy);
int gnpde_seg_softmax_f32(const int32_t* items, int64_t n_items, int64_t n_hub_items, int64_t n_long_items,
                          const int32_t* chunk_items,
                          int64_t n_chunk_items, int32_t* heavy, int64_t n_heavy, const int32_t* rowptr,
                          const int32_t* rowidx,
                          const int32_t* gidx, int group_is_dst, int out_kind, int mode, int64_t heads, int64_t dk,
                          const double* cs, const float* q, const float* k, int64_t ldqk,
                          float score_p0, float score_p1, float* w, double* m, float* rl, float* mr,
                          double* partials, void* stream);

/* Per-edge, per-head attention in COO order (the [B,E,h] `attention` that
 * SpGraphTransAttentionLayer.forward returns, function_transformer_attention.py:265-267):
 *   att[perm[p]*heads + h] = exp(s_p,h - m[g,h]) * rl[g,h]  over the aggregation CSR. */
int gnpde_edge_attention_f32(const int32_t* rowidx, const int32_t* col, const int32_t* perm, int64_t nnz,
                             int norm_idx, int mode, int64_t heads, int64_t dk,
                             const double* cs, const float* q, const float* k, int64_t ldqk,
                             float score_p0, float score_p1, const double* m, const float* rl,
                             float* att, void* stream);

/* ---------------------------------------------------------------- solver glue
 * out[i] = y0[i] + scale * sum_{j<nk} coef[j] * k_j[i]   (nk <= 8; y0 may be NULL = 0)
 * One pass for a Runge-Kutta stage input or step update (torchdiffeq
 * rk4_alt_step_func / _runge_kutta_step combinations).                      */
int gnpde_rk_combine_f32(int64_t n, const float* y0, int nk, const float* const* ks, const double* coef,
                         double scale, float* out, void* stream);

/* Entry of a solve (gnpde.integrator): dst[k] = src[order[k]] for k < rows
 * (order NULL: identity), rows of row_bytes bytes (a multiple of 16, 16-byte
 * aligned pointers); dst_copy (may be NULL) receives src unchanged,
 * dst_copy[order[k]] = src[order[k]], from the same read — the solution's
 * t0 slice and the renumbered working state in one pass.  No aliasing.      */
int gnpde_rows_copy(const void* src, int64_t rows, int64_t row_bytes, const int64_t* order, void* dst,
                    void* dst_copy, void* stream);

/* <a, b> of two fp32 arrays in fp64 (n elements), written to *out on the device:
 * the parameter gradients of the RHS backward, d alpha_train = sigma'(alpha)
 * <gf, A x - x> and d beta_train = <gf, x0> (torch autograd of
 * function_laplacian_diffusion.py:69-76).  Fixed reduction order (deterministic);
 * two launches; workspace: gnpde_dot_workspace_bytes().                      */
size_t gnpde_dot_workspace_bytes(void);
/* *out (+)= sum_i v[i] for n fp64 values (the per-row terms of the stage
 * epilogue's dot_rows), fixed order; accumulate: add to *out instead of storing.
 * Workspace gnpde_dot_workspace_bytes().                                      */
int gnpde_sum_f64(int64_t n, const double* v, double* out, int accumulate, void* workspace, size_t workspace_bytes,
                  void* stream);
int gnpde_dot_f64(int64_t n, const float* a, const float* b, double* out, void* workspace, size_t workspace_bytes,
                  void* stream);

/* The first step of an adaptive solve on the device: torchdiffeq's
 * _select_initial_step (RKAdaptiveStepsizeODESolver._before_integrate, order =
 * the tableau's order: 5 for dopri5) over n state elements, replacing the
 * Python-side torch elementwise chain and its host syncs (gnpde.integrator):
 *   scale = atol + |y0| rtol (fp32, as torch on an fp32 state)
 *   phase 0 (f1 == NULL): d0 = rms(y0/scale), d1 = rms(f0/scale),
 *     h[0] = h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 d0/d1, h[1] = d1,
 *     *hf = (float)h0 (the coef_scale of the probe y0 + h0 f0);
 *   phase 1 (f1 = f(t0 + h0, y0 + h0 f0)): d2 = rms((f1 - f0)/scale)/h0,
 *     h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? max(1e-6, 1e-3 h0) : (0.01/max(d1,d2))^(1/order),
 *     h[2] = min(100 h0, h1)  (reads h[0], h[1] of phase 0); *hf = (float)h[2] when hf
 *     is given (the first step's coef_scale, so the host need not write it).
 * Squares summed in fp64 in a fixed order (two launches per phase); h [3]
 * fp64 and hf are device memory.  Workspace gnpde_initial_step_workspace_bytes(). */
/* torchdiffeq's step-size controller after one adaptive step, on the device
 * (rk_common.py _optimal_step_size with the loop's accept test error_ratio <= 1),
 * fused with the reduction of the step's error rows (the stage epilogue's err_rows):
 *   e2    = sum_r err_rows[r]   (fixed order, as gnpde_sum_f64)
 *   ratio = sqrt(e2 / n)        (the RMS error ratio over n state elements)
 *   next  = ratio == 0 ? dt ifactor
 *         : dt min(ifactor, max(safety ratio^(-1/order), ratio < 1 ? 1 : dfactor))
 * rec[0..3] = {ratio, dt, next, e2}; *dt = next; *scale = (float)next (the
 * coef_scale of the next step's launches); t (ABI 8, NULL = none): the device
 * time of the solve, *t += dt when the step is accepted (ratio <= 1) — the step
 * start a folded dense output reads (stage dense_t).  Device pointers; two
 * launches; workspace gnpde_dot_workspace_bytes().                           */
int gnpde_adaptive_control(int64_t nrows, const double* err_rows, double n, double order, double safety,
                           double ifactor, double dfactor, double* dt, float* scale, double* rec, double* t,
                           void* workspace, size_t workspace_bytes, void* stream);
size_t gnpde_initial_step_workspace_bytes(void);
/* Phase 1 of gnpde_initial_step_f32 for an affine RHS f(y) = L y + s (ABI 8), from
 * v = L f0 (the linear part evaluated on f0, which is also the first step's u_1 / dt):
 *   d2 = rms(v / scale)   (= rms((f1 - f0)/scale)/h0 for f1 = f(y0 + h0 f0), without the
 *                          fp32 cancellation of f1 - f0)
 * then h[2] and *hf (when given) as phase 1; reads h[0], h[1] of phase 0.  scale, the
 * quotient and the fp64 squares as gnpde_initial_step_f32.  Two launches; workspace
 * gnpde_initial_step_workspace_bytes().                                        */
int gnpde_initial_step_lin_f32(int64_t n, const float* y0, const float* v, double atol, double rtol, double order,
                               double* h, float* hf, void* workspace, size_t workspace_bytes, void* stream);
int gnpde_initial_step_lin_bf16(int64_t n, const uint16_t* y0, const uint16_t* v, double atol, double rtol,
                                double order, double* h, float* hf, void* workspace, size_t workspace_bytes,
                                void* stream);
/* gnpde_initial_step_f32's scalar rules from per-row squared sums formed by the RHS
 * launches themselves (ABI 8; an affine RHS f(y) = L y + s): phase 0 (rows_b given)
 * with rows_a = the f0 launch's err_rows (e = f0, err_y1 = -2: sum (f0/scale)^2) and
 * rows_b = its scale_rows (sum (y0/scale)^2); phase 1 (rows_b NULL) with rows_a =
 * the err_rows of a launch evaluating L f0 (the linear part on f0, e = f): then
 *   d2 = rms(L f0 / scale)   (= rms((f1 - f0)/scale)/h0 for f1 = f(y0 + h0 f0))
 * and h[2], *hf as gnpde_initial_step_f32's phase 1.  scale = atol + rtol |y0| in
 * fp64 (the epilogue's tolerance), n the state's element count.  Two launches;
 * workspace gnpde_initial_step_workspace_bytes().                             */
int gnpde_initial_step_rows(int64_t nrows, const double* rows_a, const double* rows_b, double n, double order,
                            double* h, float* hf, void* workspace, size_t workspace_bytes, void* stream);
/* The squared sums of gnpde_initial_step_f32 without its scalar rules (ABI 7): the
 * per-component pieces of a mixed norm (torchdiffeq's adjoint norm: the max over the
 * components [y | adj_y | adj_params] of their RMS norms), the caller combining them:
 *   f1 == NULL: out[0] = sum (y0/scale)^2, out[1] = sum (f0/scale)^2
 *   else:       out[0] = sum ((f1 - f0)/scale)^2, out[1] = 0
 * scale = atol + |y0| rtol in fp32, squares in fp64, the fixed order of
 * gnpde_initial_step_f32.  Workspace gnpde_initial_step_workspace_bytes().     */
int gnpde_scaled_sq_sums_f32(int64_t n, const float* y0, const float* f0, const float* f1, double atol, double rtol,
                             double* out, void* workspace, size_t workspace_bytes, void* stream);
/* out[s] = sum_{i < len} v[s*len + i] for s < nseg (ABI 7): the row sums of several
 * epilogue channels of one adaptive step (the y and adjoint error rows, the alpha
 * integrand's rows of every stage) in one pass, each in a fixed order
 * (deterministic).  Workspace gnpde_segment_sums_workspace_bytes(nseg).        */
size_t gnpde_segment_sums_workspace_bytes(int64_t nseg);
int gnpde_segment_sums_f64(int64_t nseg, int64_t len, const double* v, double* out, void* workspace,
                           size_t workspace_bytes, void* stream);
int gnpde_initial_step_f32(int64_t n, const float* y0, const float* f0, const float* f1, double atol, double rtol,
                           double order, double* h, float* hf, void* workspace, size_t workspace_bytes, void* stream);
int gnpde_initial_step_bf16(int64_t n, const uint16_t* y0, const uint16_t* f0, const uint16_t* f1, double atol,
                            double rtol, double order, double* h, float* hf, void* workspace, size_t workspace_bytes,
                            void* stream);

/* ---------------------------------------------------------------- backward
 * Gradients of the RHS f = a (A(w) x - x) [+ b x0] and of the attention that
 * produces w; torch autograd of the reference (function_laplacian_diffusion.py:
 * 39-77, function_transformer_attention.py:218-267, utils.py:116-127) restated
 * as graph passes.  All sums in a fixed order (no float atomics).
 *
 * d f / d w: g_out[perm[p]*heads + h] = a * <gf[rowidx[p]], x[col[p]]> / heads
 * for every head h < heads <= 64 (COO order; heads > 1: w is the head mean of [B,E,heads]).
 * a = sigmoid(*alpha) / *alpha / 1 (alpha NULL), as the RHS epilogue.        */
int gnpde_sddmm_f32(const int32_t* rowidx, const int32_t* col, const int32_t* perm, int64_t nnz, int64_t C,
                    const float* gf, int64_t ldg, const float* x, int64_t ldx, const float* alpha, int alpha_sigmoid,
                    int heads, float* g_out, void* stream);

/* Edge-softmax backward per group of a grouped CSR (rowptr, perm -> COO ids):
 * gs[i,h] = att[i,h] * (g[i,h] - sum_{j in grp(i)} att[j,h] g[j,h]), COO [nnz, heads]. */
int gnpde_softmax_backward_f32(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, int heads,
                               const float* att, const float* g, float* gs, void* stream);

/* out[r,h] = sum_{p in row r} vals[perm[p]*heads + h]  (fp64 out, [R, heads]). */
int gnpde_segment_sum_f64(const int32_t* rowptr, const int32_t* perm, int64_t R, int64_t nnz, int heads,
                          const float* vals, double* out, void* stream);

/* y[b][h][c] = sum_n w[b*N+n, h] x[b*N+n, c], y[b][h][C] = sum_n w[b*N+n, h]
 * (fp64, y is [B][heads][C+1]); workspace gnpde_wcolsum_workspace_bytes.    */
size_t gnpde_wcolsum_workspace_bytes(int64_t B, int64_t N, int64_t C, int heads);
int gnpde_wcolsum_f64(const float* x, int64_t B, int64_t N, int64_t C, int64_t ldx, const double* w, int heads,
                      double* y, void* workspace, size_t workspace_bytes, void* stream);

/* Input gradient of the reference-mode node scores cs = x U_b + v_b and of the
 * key sum xbar_b = sum_n deg[n] x_n:
 *   gx[n,c] (+)= sum_h gcs[n,h] U[b][c][h] + deg[n] gxbar[b][c]   (b = n / N). */
int gnpde_score_input_grad_f32(const double* gcs, const double* U, const int32_t* deg, const double* gxbar, int64_t B,
                               int64_t N, int64_t C, int heads, float* gx, int64_t ldgx, int accumulate,
                               void* stream);

/* out[p] = scale * w[perm[p]*heads + h]: one head of COO per-edge values in a
 * grouped CSR's order (per-head weights of the per-edge score backward).     */
int gnpde_gather_head_f32(const float* w, int64_t nnz, int heads, int h, const int32_t* perm, float scale, float* out,
                          void* stream);

/* Backward of the per-edge scores (SCORE_DOT / EXP_KERNEL / COSINE / PEARSON,
 * function_transformer_attention.py:246-259) onto the projections: over a
 * grouped CSR whose rows receive the gradient (side 0: the aggregation CSR,
 * rows = sources, own operand q; side 1: the CSC, rows = destinations, own k;
 * col = the other endpoint, perm -> COO ids), with gs [E, heads] = dL/ds in
 * COO order:
 *   out[r, h*dk + d] = sum_{e in row r} gs[e,h] * ds_e,h / d own[r, h*dk + d]
 * (out [R, ldo], overwritten; fixed order, deterministic).  For EXP_KERNEL and
 * gp != NULL also gp[e*2H + h] = gs * ds/d(output_var), gp[e*2H + H + h] =
 * gs * ds/d(lengthscale) (COO order; the caller sums them).  attention_dim
 * <= 1024.                                                                   */
int gnpde_score_grad_f32(const int32_t* rowptr, const int32_t* col, const int32_t* perm, int64_t R, int64_t nnz,
                         int side, int mode, int64_t heads, int64_t dk, const float* q, const float* k, int64_t ldqk,
                         float score_p0, float score_p1, const float* gs, float* out, int64_t ldo, float* gp,
                         void* stream);

#ifdef __cplusplus
}
#endif
#endif /* GNPDE_H_ */
