// common.hpp — shared helpers for the gnpde HIP kernels (gfx950 / CDNA4, wave64).
#pragma once
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <string>

#include "../../include/gnpde.h"

// Experiment builds (make EXPERIMENTS=1): the A/B knobs of the round-1/2 sweeps
// (environment-selected K1 geometries, the separate hub fixup launch, the
// XCD remap, the bf16 vector cap).  The product library is built without them.
#ifndef GNPDE_EXPERIMENTS
#define GNPDE_EXPERIMENTS 0
#endif

namespace gnpde {

// ------------------------------------------------------------------ error plumbing
void set_error(const char* fmt, ...);

#define GNPDE_REQUIRE(cond, code, ...)      \
  do {                                      \
    if (!(cond)) {                          \
      ::gnpde::set_error(__VA_ARGS__);      \
      return (code);                        \
    }                                       \
  } while (0)

#define GNPDE_HIP(call)                                                                 \
  do {                                                                                  \
    hipError_t e_ = (call);                                                             \
    if (e_ != hipSuccess) {                                                             \
      ::gnpde::set_error("%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                         __LINE__);                                                     \
      return GNPDE_EHIP;                                                                \
    }                                                                                   \
  } while (0)

#define GNPDE_LAUNCH_CHECK() GNPDE_HIP(hipGetLastError())

inline hipStream_t as_stream(void* s) { return reinterpret_cast<hipStream_t>(s); }

inline bool aligned16(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 15u) == 0; }
inline bool aligned8(const void* p) { return (reinterpret_cast<uintptr_t>(p) & 7u) == 0; }

constexpr int kWave = 64;          // CDNA wavefront width
constexpr int kBlock = 256;        // 4 waves per workgroup
constexpr int kWavesPerBlock = kBlock / kWave;
constexpr float kSoftmaxEps = 1e-16f;  // utils.softmax denominator epsilon, src/utils.py:124-125
// Packed statistics record of one softmax group (optional output of the
// statistics kernels, read by the fused-weight K1 with one load per edge):
// H floats m[h] (the group max rounded to fp32; the sum is taken relative to
// it), then H floats rl[h], padded to 16 bytes — 16 B for two heads.
__host__ __device__ constexpr int stats_record_floats(int H) { return (2 * H + 3) & ~3; }

// ------------------------------------------------------------------ vector loads
template <int VEC>
__device__ __forceinline__ void load_vec(const float* __restrict__ p, float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    const float4 u = *reinterpret_cast<const float4*>(p + 4);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
    v[4] = u.x; v[5] = u.y; v[6] = u.z; v[7] = u.w;
  } else if constexpr (VEC == 4) {
    const float4 t = *reinterpret_cast<const float4*>(p);
    v[0] = t.x; v[1] = t.y; v[2] = t.z; v[3] = t.w;
  } else if constexpr (VEC == 2) {
    const float2 t = *reinterpret_cast<const float2*>(p);
    v[0] = t.x; v[1] = t.y;
  } else {
    v[0] = *p;
  }
}

template <int VEC>
__device__ __forceinline__ void store_vec(float* __restrict__ p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
  } else if constexpr (VEC == 4) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<float2*>(p) = make_float2(v[0], v[1]);
  } else {
    *p = v[0];
  }
}

// bf16 storage (configs[3]): rows are stored as bfloat16, every sum and the
// epilogue run in fp32; stores round to nearest even (as torch's .to(bfloat16)).
struct bf16 {
  uint16_t bits;
};

__device__ __forceinline__ float bf16_to_f32(uint32_t b) { return __uint_as_float(b << 16); }

__device__ __forceinline__ uint32_t f32_to_bf16(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (u >> 16) | 0x40u;  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return u >> 16;
}

template <int VEC>
__device__ __forceinline__ void load_vec(const bf16* __restrict__ p, float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    const uint32_t w[4] = {t.x, t.y, t.z, t.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      v[2 * i] = bf16_to_f32(w[i] & 0xffffu);
      v[2 * i + 1] = bf16_to_f32(w[i] >> 16);
    }
  } else if constexpr (VEC == 4) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    v[0] = bf16_to_f32(t.x & 0xffffu); v[1] = bf16_to_f32(t.x >> 16);
    v[2] = bf16_to_f32(t.y & 0xffffu); v[3] = bf16_to_f32(t.y >> 16);
  } else if constexpr (VEC == 2) {
    const uint32_t t = *reinterpret_cast<const uint32_t*>(p);
    v[0] = bf16_to_f32(t & 0xffffu); v[1] = bf16_to_f32(t >> 16);
  } else {
    v[0] = bf16_to_f32(p->bits);
  }
}

template <int VEC>
__device__ __forceinline__ void store_vec(bf16* __restrict__ p, const float (&v)[VEC]) {
  if constexpr (VEC == 8) {
    uint4 t;
    t.x = f32_to_bf16(v[0]) | (f32_to_bf16(v[1]) << 16);
    t.y = f32_to_bf16(v[2]) | (f32_to_bf16(v[3]) << 16);
    t.z = f32_to_bf16(v[4]) | (f32_to_bf16(v[5]) << 16);
    t.w = f32_to_bf16(v[6]) | (f32_to_bf16(v[7]) << 16);
    *reinterpret_cast<uint4*>(p) = t;
  } else if constexpr (VEC == 4) {
    uint2 t;
    t.x = f32_to_bf16(v[0]) | (f32_to_bf16(v[1]) << 16);
    t.y = f32_to_bf16(v[2]) | (f32_to_bf16(v[3]) << 16);
    *reinterpret_cast<uint2*>(p) = t;
  } else if constexpr (VEC == 2) {
    *reinterpret_cast<uint32_t*>(p) = f32_to_bf16(v[0]) | (f32_to_bf16(v[1]) << 16);
  } else {
    p->bits = (uint16_t)f32_to_bf16(v[0]);
  }
}

__device__ __forceinline__ int uniform(int v) { return __builtin_amdgcn_readfirstlane(v); }

typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

// ------------------------------------------------------------------ buffer memory ops
// Raw buffer loads/stores take a 32-bit byte offset from a wave-uniform base,
// and the hardware drops an access at or past num_records: a lane with nothing
// to load or store passes kBufNone, so predicated accesses need no branch.
// That matters on gfx9, where stores count in vmcnt: a store under a branch
// makes the compiler's later waits conservative (vmcnt(0)), which serialises
// every following store and load behind it.  Byte offsets must stay below
// kBufRecords (callers check their buffer sizes).
constexpr uint32_t kBufRecords = 0xffffff00u;
constexpr uint32_t kBufNone = 0xfffffff0u;
constexpr int kWaitVm0 = 0x0f70;  // s_waitcnt vmcnt(0) (expcnt, lgkmcnt at max)

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* p) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), 0, (int)kBufRecords, 0x00020000);
}
__device__ __forceinline__ void buf_store_f32(__amdgpu_buffer_rsrc_t r, uint32_t off, float v) {
  __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v), r, off, 0, 0);
}
__device__ __forceinline__ void buf_store_f64(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, 0);
}


// butterfly reductions over the 64 lanes of a wavefront
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ double wave_max(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o));
  return v;
}
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}
__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
  return v;
}

// RHS epilogue scalars (device scalars: no host sync, graph-capturable)
// Workgroups are dispatched round-robin over the 8 XCDs (workgroup b runs on
// XCD b % 8).  With remap on, XCD x is handed one contiguous run of the grid's
// work instead of every 8th workgroup, so rows handled together share an L2.
constexpr int kNumXcd = 8;
__device__ __forceinline__ int xcd_block(int remap) {
  const int b = blockIdx.x;
  if (!remap) return b;
  const int nb = gridDim.x;
  const int x = b % kNumXcd, k = b / kNumXcd;
  if (remap >= 2) {
    // chunks of `remap` consecutive blocks, chunk i on XCD i % 8: each XCD walks
    // runs of neighbouring items (L2 locality) while every XCD still samples
    // every part of the item list (load balance).  Blocks past the last whole
    // round of chunks keep the hardware's order.
    const int K = remap, round = K * kNumXcd;
    const int whole = nb / round * round;
    if (b >= whole) return b;
    return ((k / K) * kNumXcd + x) * K + (k % K);
  }
  const int q = nb / kNumXcd, r = nb % kNumXcd;
  return x < r ? x * (q + 1) + k : r * (q + 1) + (x - r) * q + k;
}

struct Epi {
  int xcd_remap;
  const float* x;
  int64_t ldx;
  const float* x0;
  int64_t ldx0;
  const float* alpha;
  const float* beta;
  int flags;
  float* f;
  int64_t ldf;
  int has_stage;
  gnpde_stage_epilogue_t st;
};

__device__ __forceinline__ float epi_alpha(const Epi& e) {
  const float a = *e.alpha;
  return (e.flags & GNPDE_ALPHA_SIGMOID) ? 1.0f / (1.0f + expf(-a)) : a;
}

// Epilogue operands of one row slice, loaded ahead of the aggregation so their
// latency overlaps the gathers (they depend only on the row).
// A row slice kept in its storage form (VEC elements of T as raw dwords) until
// it is used: bf16 operands held across the gather loop cost half the
// registers of their fp32 conversion.
template <int VEC, class T>
struct Packed {
  static constexpr int W = (VEC * (int)sizeof(T) + 3) / 4;
  uint32_t d[W];
};

template <int VEC>
__device__ __forceinline__ void load_packed(const float* __restrict__ p, Packed<VEC, float>& r) {
  float v[VEC];
  load_vec<VEC>(p, v);
#pragma unroll
  for (int i = 0; i < VEC; ++i) r.d[i] = __float_as_uint(v[i]);
}

template <int VEC>
__device__ __forceinline__ void load_packed(const bf16* __restrict__ p, Packed<VEC, bf16>& r) {
  if constexpr (VEC == 8) {
    const uint4 t = *reinterpret_cast<const uint4*>(p);
    r.d[0] = t.x; r.d[1] = t.y; r.d[2] = t.z; r.d[3] = t.w;
  } else if constexpr (VEC == 4) {
    const uint2 t = *reinterpret_cast<const uint2*>(p);
    r.d[0] = t.x; r.d[1] = t.y;
  } else if constexpr (VEC == 2) {
    r.d[0] = *reinterpret_cast<const uint32_t*>(p);
  } else {
    r.d[0] = p->bits;
  }
}

template <int VEC>
__device__ __forceinline__ float unpack(const Packed<VEC, float>& r, int t) {
  return __uint_as_float(r.d[t]);
}

template <int VEC>
__device__ __forceinline__ float unpack(const Packed<VEC, bf16>& r, int t) {
  return bf16_to_f32((t & 1) ? (r.d[t >> 1] >> 16) : (r.d[t >> 1] & 0xffffu));
}

// ------------------------------------------------------------------ streamed stage operands
// The operand rows of the streamed stage epilogues (STG 4, the non-prefetching
// STG 1-3, gnpde_stage_apply_*) are ISSUED TOGETHER, before any of them is used:
// one memory round trip per epilogue.  Written as "if (j < nk) { load k[j];
// fma }" the compiler waits for each load before the next (one round trip per
// operand: the G-arxiv dopri5 launches with 3-6 operands ran at 172 us against
// 92 us for the rk4 stage, round 4).  The loads are raw buffer loads whose absent
// operands take the out-of-range offset kBufNone (no memory access, value 0),
// so nothing in the load sequence branches.  Buffer byte offsets are 32-bit: a
// wavefront any of whose rows lies past 4 GiB of the state takes the per-operand
// form.
// GNPDE_WIDE_BATCH=0 builds the per-operand form (A/B only).
#ifndef GNPDE_WIDE_BATCH
#define GNPDE_WIDE_BATCH 1
#endif
#ifndef GNPDE_WIDE_NOFB
#define GNPDE_WIDE_NOFB 0
#endif
#ifndef GNPDE_STG4_PRE
#define GNPDE_STG4_PRE 0  // wide-epilogue operand rows read before the gathers (A/B)
#endif

template <int VEC, class T>
__device__ __forceinline__ void buf_load_packed(const void* p, uint32_t boff, Packed<VEC, T>& r) {
  const __amdgpu_buffer_rsrc_t rs = buf_rsrc(p);
  constexpr int B = VEC * (int)sizeof(T);
  if constexpr (B == 32) {
    // a dropped load (kBufNone) stays dropped: kBufNone + 16 would wrap to offset 0
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 0);
    const u32x4 u = __builtin_amdgcn_raw_buffer_load_b128(rs, boff >= kBufRecords ? kBufNone : boff + 16u, 0, 0);
    r.d[0] = v.x;
    r.d[1] = v.y;
    r.d[2] = v.z;
    r.d[3] = v.w;
    r.d[4] = u.x;
    r.d[5] = u.y;
    r.d[6] = u.z;
    r.d[7] = u.w;
  } else if constexpr (B == 16) {
    const u32x4 v = __builtin_amdgcn_raw_buffer_load_b128(rs, boff, 0, 0);
    r.d[0] = v.x;
    r.d[1] = v.y;
    r.d[2] = v.z;
    r.d[3] = v.w;
  } else if constexpr (B == 8) {
    const u32x2 v = __builtin_amdgcn_raw_buffer_load_b64(rs, boff, 0, 0);
    r.d[0] = v.x;
    r.d[1] = v.y;
  } else if constexpr (B == 4) {
    r.d[0] = __builtin_amdgcn_raw_buffer_load_b32(rs, boff, 0, 0);
  } else {
    static_assert(B == 2, "row slices are 2-16 bytes");
    r.d[0] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b16(rs, boff, 0, 0);
  }
}

// An operand row slice, or zeros for an absent operand (p == NULL, wave-uniform):
// GNPDE_WIDE_SKIP=1 skips the absent operand's load under a scalar branch (an
// out-of-range buffer load still costs an address-unit pass over the wavefront);
// the waits stay at the first use after the whole batch.
#ifndef GNPDE_WIDE_SKIP
#define GNPDE_WIDE_SKIP 1
#endif
template <int VEC, class T>
__device__ __forceinline__ void opt_load(const float* p, uint32_t bo, Packed<VEC, T>& r) {
  if (GNPDE_WIDE_SKIP) {
    if (p) {
      buf_load_packed<VEC, T>(p, bo, r);
    } else {
#pragma unroll
      for (int t = 0; t < Packed<VEC, T>::W; ++t) r.d[t] = 0u;
    }
  } else {
    buf_load_packed<VEC, T>(p, p ? bo : kBufNone, r);
  }
}

// Whether every row of the wavefront addresses the state with 32-bit buffer offsets
template <int VEC, class T>
__device__ __forceinline__ bool rows_fit_buffer(int64_t off) {
  return __all((off + VEC) * (int64_t)sizeof(T) < (int64_t)kBufRecords);
}

// The operand slots of the wide epilogue, in consumption order: the NOUT output
// bases, the error base, k[0..NKMAX-1], the error tolerance's y0 (ERR).  p[q] is
// NULL for an absent operand or one equal to the RHS input xid (its values are
// already held); cb the bases' coefficients (0 without a base).
template <int NOUT, int NKMAX, bool ERR>
struct WideSlots {
  static constexpr int N = NOUT + NKMAX + (ERR ? 2 : 0);
  const float* p[N];
  float cb[NOUT + 1];
  // the slot id of position q (slot ids: bases 0..NOUT-1, k rows NOUT + j, error base
  // NOUT + NKMAX, y0 N - 1 — as the consumers below number them)
  __device__ static constexpr int slot(int q) {
    return q < NOUT ? q : (ERR && q == NOUT ? NOUT + NKMAX : (q < NOUT + (ERR ? 1 : 0) + NKMAX ? q - (ERR ? 1 : 0) : N - 1));
  }
};

template <int NOUT, int NKMAX, bool ERR>
__device__ __forceinline__ void wide_slots(const gnpde_stage_epilogue_t& st, const float* xid,
                                           WideSlots<NOUT, NKMAX, ERR>& w) {
  const bool has_err = ERR && st.err_rows != nullptr;
#pragma unroll
  for (int i = 0; i <= NOUT; ++i) {
    if (i == NOUT && !ERR) break;
    const bool on = i < NOUT ? i < st.n_out : has_err;
    const gnpde_stage_out_t& so = i < NOUT ? st.o[i] : st.err;
    const float* b = on ? so.base : nullptr;
    w.cb[i] = b ? so.cb : 0.f;
    w.p[i] = (b && b != xid) ? b : nullptr;  // position i: output bases, then the error base
  }
#pragma unroll
  for (int j = 0; j < NKMAX; ++j) w.p[NOUT + (ERR ? 1 : 0) + j] = (j < st.nk && st.k[j] != xid) ? st.k[j] : nullptr;
  if constexpr (ERR) {
    // the tolerance's y0: not loaded again when it is a loaded output base (wide_combine copies it)
    bool dup = false;
#pragma unroll
    for (int i = 0; i < NOUT; ++i) dup = dup || (w.p[i] != nullptr && w.p[i] == st.err_y0);
    // (nor when it is the RHS input: its values are held, wide_combine packs them)
    w.p[WideSlots<NOUT, NKMAX, ERR>::N - 1] = (has_err && !dup && st.err_y0 != xid) ? st.err_y0 : nullptr;
  }
}

// fp32 values -> a row slice in storage form (bf16: round to nearest even); for an
// operand that equals the RHS input, whose values are already fp32-exact in T
template <int VEC, class T>
__device__ __forceinline__ void pack_into(const float (&v)[VEC], Packed<VEC, T>& r) {
  if constexpr (sizeof(T) == 4) {
#pragma unroll
    for (int i = 0; i < VEC; ++i) r.d[i] = __float_as_uint(v[i]);
  } else {
#pragma unroll
    for (int i = 0; i < VEC; ++i) {
      const uint32_t b = f32_to_bf16(v[i]);
      r.d[i >> 1] = (i & 1) ? (r.d[i >> 1] | (b << 16)) : b;
    }
  }
}

// Epilogue operands of one row slice, loaded ahead of the aggregation so their
// latency overlaps the gathers (they depend only on the row).
// STG = the stage epilogue an instantiation is compiled for:
//   0: store f;
//   1: one stage output, at most kStagePre shared operands, no dot / error term
//      (every fixed-grid step of gnpde.integrator);
//   3: one output plus the dot term (its operand loaded in the epilogue: the
//      adjoint stages that emit one combination);
//   2: the general fixed-grid epilogue (two outputs, dot term);
//   4: the wide epilogue of the adaptive solvers: two outputs, up to
//      GNPDE_STAGE_MAX_K operands and the embedded pair's error rows, every stage
//      operand loaded after the aggregation (nothing held across the gathers);
//   5: the wide epilogue plus the step's folded dense output (ABI 8 dense_out: the
//      last launch of an affine Krylov step that may cross an output time).
// An instantiation only holds registers for what it can emit.
constexpr int kStagePre = 2;
template <int STG>
constexpr bool stage_wide() {
  return STG == 4 || STG == 5;
}
// A/B knobs: whether the STG 1 / 2 / 3 instantiations prefetch their stage
// operands before the gathers (1) or stream them after the aggregation (0, as STG 4)
#ifndef GNPDE_STG1_PRE
#define GNPDE_STG1_PRE 1
#endif
#ifndef GNPDE_STG2_PRE
#define GNPDE_STG2_PRE 0  // 111 -> 69 VGPRs (4 -> 7 waves per SIMD)
#endif
#ifndef GNPDE_STG3_PRE
#define GNPDE_STG3_PRE 0  // G-arxiv adjoint launch (CSC): 134 with, 117 us without (105 -> fewer VGPRs)
#endif
#ifndef GNPDE_DOT_PRE
#define GNPDE_DOT_PRE 1   // the dot operand and the row's running dot read before the gathers: 128 -> 117 us
#endif
#ifndef GNPDE_DOT_DIAG
#define GNPDE_DOT_DIAG 0  // diagnostics only (wrong results): 1 no dot arithmetic, 2 no row reduction / store
#endif
#ifndef GNPDE_ERR_DIAG
#define GNPDE_ERR_DIAG 0  // diagnostics only (wrong results): bit 1 no error-term arithmetic, bit 2 no row sum
// (G-arxiv K1 with error rows and no output, round 6: 116 us; bit 1: 106; bit 2: 91 — the per-row
// error sum at the end of every wave costs ~20 us of a launch; whole-granule row stores: no change)
#endif
#ifndef GNPDE_STG2_DW
#define GNPDE_STG2_DW 1   // STG 2 prefetches its dot operand too (with GNPDE_DOT_PRE)
#endif
template <int STG>
constexpr int stage_nout() {
  return (STG == 2 || stage_wide<STG>()) ? 2 : 1;
}
template <int STG>
constexpr bool stage_prefetch() {
  return (STG == 1 && GNPDE_STG1_PRE) || (STG == 2 && GNPDE_STG2_PRE) || (STG == 3 && GNPDE_STG3_PRE);
}
template <int STG>
constexpr int stage_kpre() {  // operands prefetched before the gathers
  return stage_prefetch<STG>() ? kStagePre : 0;
}
template <int STG>
constexpr int stage_bpre() {  // stage-output bases prefetched before the gathers
  return stage_prefetch<STG>() ? stage_nout<STG>() : 0;
}
template <int STG>
constexpr bool stage_dot() {
  return STG == 2 || STG == 3;
}
template <int STG>
constexpr bool stage_dw_pre() {  // the dot operand read before the gathers
  return (STG == 2 && (stage_prefetch<STG>() || (GNPDE_DOT_PRE && GNPDE_STG2_DW))) || (STG == 3 && GNPDE_DOT_PRE);
}
template <int STG>
constexpr bool stage_err() {
  return stage_wide<STG>();
}

template <int VEC, class T, int STG>
struct EpiPre {
  Packed<VEC, T> xr;
  Packed<VEC, T> x0r;
  Packed<VEC, T> base[stage_bpre<STG>() > 0 ? stage_bpre<STG>() : 1];
  Packed<VEC, T> kv[stage_kpre<STG>() > 0 ? stage_kpre<STG>() : 1];
  Packed<VEC, T> dw;  // the stage's dot operand (dot_rows; STG 2 with GNPDE_STG2_PRE, STG 3 with GNPDE_DOT_PRE)
  double dprev;       // the row's running dot (dot_accumulate), read before the gathers
  Packed<VEC, T> wk[(stage_wide<STG>() && GNPDE_STG4_PRE > 0) ? GNPDE_STG4_PRE : 1];  // the wide epilogue's first operands
};

// The Epi / stage pointers are declared float*; for bf16 storage they address
// bf16 arrays (gnpde_spmm_rhs_bf16) and are read through T.
template <class T>
__device__ __forceinline__ const T* as_t(const float* p) {
  return reinterpret_cast<const T*>(p);
}
template <class T>
__device__ __forceinline__ T* as_t(float* p) {
  return reinterpret_cast<T*>(p);
}

template <int VEC, int STG, class T = float>
__device__ __forceinline__ void epi_prefetch(const Epi& e, int64_t row, int cc, EpiPre<VEC, T, STG>& p) {
  const bool need_x = (e.flags & GNPDE_EPI_RHS) != 0;
  if (need_x) load_packed<VEC>(as_t<T>(e.x) + row * e.ldx + cc, p.xr);
  if (e.flags & GNPDE_ADD_SOURCE) load_packed<VEC>(as_t<T>(e.x0) + row * e.ldx0 + cc, p.x0r);
  if constexpr (stage_dot<STG>() && GNPDE_DOT_PRE)  // the running dot: its read is off the epilogue's chain
    p.dprev = (e.st.dot_rows && e.st.dot_accumulate) ? e.st.dot_rows[row] : 0.0;
  if constexpr (stage_wide<STG>() && GNPDE_STG4_PRE > 0) {
    // the first GNPDE_STG4_PRE present operand rows of the wide epilogue (WideSlots order)
    const int64_t off = row * e.ldf + cc;
    if (GNPDE_WIDE_BATCH && rows_fit_buffer<VEC, T>(off)) {
      WideSlots<2, GNPDE_STAGE_MAX_K, true> w;
      wide_slots<2, GNPDE_STAGE_MAX_K, true>(e.st, (need_x && e.ldx == e.ldf) ? e.x : nullptr, w);
      const uint32_t bo = (uint32_t)(off * (int64_t)sizeof(T));
      int cnt = 0;
#pragma unroll
      for (int q = 0; q < WideSlots<2, GNPDE_STAGE_MAX_K, true>::N; ++q) {
        if (w.p[q]) {
#pragma unroll
          for (int c = 0; c < GNPDE_STG4_PRE; ++c)
            if (cnt == c) buf_load_packed<VEC, T>(w.p[q], bo, p.wk[c]);
          ++cnt;
        }
      }
    }
  }
  if constexpr (STG == 0 || stage_wide<STG>()) return;
  const int64_t off = row * e.ldf + cc;
#pragma unroll
  for (int i = 0; i < stage_bpre<STG>(); ++i) {
    if (i < e.st.n_out) {
      const gnpde_stage_out_t& so = e.st.o[i];
      if (so.base != nullptr && !(need_x && so.base == e.x && e.ldx == e.ldf))
        load_packed<VEC>(as_t<T>(so.base) + off, p.base[i]);
    }
  }
#pragma unroll
  for (int j = 0; j < stage_kpre<STG>(); ++j)
    if (j < e.st.nk && !(need_x && e.st.k[j] == e.x && e.ldx == e.ldf)) load_packed<VEC>(as_t<T>(e.st.k[j]) + off, p.kv[j]);
  // the dot operand: STG 2 when prefetching, STG 2 / 3 under GNPDE_DOT_PRE (else in the epilogue)
  if constexpr (stage_dw_pre<STG>())
    if (e.st.dot_rows) load_packed<VEC>(as_t<T>(e.st.dot_with) + off, p.dw);
}

// One stage combination cb*base + sc*cf*f + sum_j sc*c[j]*k[j] of a row slice
// (sc = *coef_scale or 1; multiplying by 1.0f changes no bit).  The base is x
// (already in registers), a prefetched row (pre != nullptr) or loaded here.
template <int VEC, int NK, class T, class KV>
__device__ __forceinline__ void stage_combine(const Epi& e, const gnpde_stage_out_t& so, int64_t off,
                                              const float (&o)[VEC], const Packed<VEC, T>& xr,
                                              const Packed<VEC, T>* pre, const KV& kval, float sc, float (&r)[VEC]) {
  const bool need_x = (e.flags & GNPDE_EPI_RHS) != 0;
  if (so.base == nullptr) {
#pragma unroll
    for (int t = 0; t < VEC; ++t) r[t] = 0.f;
  } else if (need_x && so.base == e.x && e.ldx == e.ldf) {
#pragma unroll
    for (int t = 0; t < VEC; ++t) r[t] = so.cb * unpack(xr, t);
  } else {
    Packed<VEC, T> bv;
    if (pre)
      bv = *pre;
    else
      load_packed<VEC>(as_t<T>(so.base) + off, bv);
#pragma unroll
    for (int t = 0; t < VEC; ++t) r[t] = so.cb * unpack(bv, t);
  }
#pragma unroll
  for (int j = 0; j < NK; ++j) {
    if (j < e.st.nk) {
      const float c = so.c[j] * sc;
#pragma unroll
      for (int t = 0; t < VEC; ++t) r[t] = fmaf(c, kval(j, t), r[t]);
    }
  }
  const float cf = so.cf * sc;
#pragma unroll
  for (int t = 0; t < VEC; ++t) r[t] = fmaf(cf, o[t], r[t]);
}

__device__ __forceinline__ float stage_scale(const gnpde_stage_epilogue_t& st) {
  return st.coef_scale ? *st.coef_scale : 1.f;
}

// output i's coefficient scale: sc, or 1 when its bit in unscaled_outs is set (ABI 6)
__device__ __forceinline__ float out_scale(const gnpde_stage_epilogue_t& st, int i, float sc) {
  return (st.unscaled_outs >> i) & 1 ? 1.f : sc;
}

// The folded dense output of an adaptive step (ABI 8 dense_out, STG 5): whether the
// step crosses the output time, and the fp32 coefficients of its operands — [0] the
// base of output 0 (y0), [1 + j] k[j], [GNPDE_STAGE_MAX_K + 1] f — formed in fp64
// from the device step start, output time and step size by dense_coef_kernel (one
// wavefront ahead of the launch) into dense_tab = {crossing, c[0..7]}, which the
// launch reads into scalar registers (wave-uniform values).
constexpr int kDenseSlots = GNPDE_STAGE_MAX_K + 2;
struct DenseCoef {
  bool on;
  float c[kDenseSlots];
};

__device__ __forceinline__ DenseCoef dense_load(const gnpde_stage_epilogue_t& st) {
  DenseCoef d;
  const float* tab = st.dense_tab;
  d.on = __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, tab[0])) != 0;
#pragma unroll
  for (int q = 0; q < kDenseSlots; ++q)
    d.c[q] = __builtin_bit_cast(float, __builtin_amdgcn_readfirstlane(__builtin_bit_cast(int, tab[1 + q])));
  return d;
}

__device__ __forceinline__ void dense_coefs(const gnpde_stage_epilogue_t& st, float* tab) {
  const double t0 = st.dense_t[0], tout = st.dense_t[1], h = *st.dense_dt;
  const bool on = t0 < tout && tout <= t0 + h;
  const double x = on ? (tout - t0) / h : 0.0;
  const double x2 = x * x, x3 = x2 * x, x4 = x2 * x2;
  const double cy0 = 1.0 - 11.0 * x2 + 18.0 * x3 - 8.0 * x4;
  const double cy1 = -5.0 * x2 + 14.0 * x3 - 8.0 * x4;
  const double cym = 16.0 * x2 - 32.0 * x3 + 16.0 * x4;
  const double w[GNPDE_DENSE_BASIS] = {cy0 + cy1 + cym, h * cy1, h * cym, h * (x - 4.0 * x2 + 5.0 * x3 - 2.0 * x4),
                                       h * (x2 - 3.0 * x3 + 2.0 * x4)};
  tab[0] = __builtin_bit_cast(float, on ? 1 : 0);
#pragma unroll
  for (int q = 0; q < kDenseSlots; ++q) {
    double c = 0.0;
#pragma unroll
    for (int m = 0; m < GNPDE_DENSE_BASIS; ++m) c = fma(w[m], (double)st.dense_m[m][q], c);
    tab[1 + q] = (float)c;
  }
}

// The wide stage epilogue of one row slice (STG 4; also gnpde_stage_apply_*):
// every output and the error combination start from cb*base (x when the base is
// the RHS input xid, with values xv), take sc*c[j]*k[j] for j ascending, then
// sc*cf*f — per output the same order as stage_combine, so the same bits.
// Returns the error combination in ev (when err_rows), output values in r and,
// when y0v is given and err_rows is set, the tolerance's y0 row slice.  DENSE (STG
// 5): also the dense output sum_q dc[q] * operand q in rd (base of output 0, k[j], f).
template <int VEC, class T, int NKMAX = GNPDE_STAGE_MAX_K, int NOUT = 2, bool ERR = true, int PK = 0,
          bool DENSE = false>
__device__ __forceinline__ void wide_combine(const gnpde_stage_epilogue_t& st, int64_t off, const float (&o)[VEC],
                                             const float* xid, const float (&xv)[VEC], float (&r)[2][VEC],
                                             float (&ev)[VEC], Packed<VEC, T>* y0v = nullptr,
                                             const Packed<VEC, T>* pre = nullptr, const float* dc = nullptr,
                                             float* rd = nullptr) {
  const float sc = stage_scale(st);
  float sco[NOUT];  // the outputs' coefficient scales (the error term's is sc)
#pragma unroll
  for (int i = 0; i < NOUT; ++i) sco[i] = out_scale(st, i, sc);
  if (GNPDE_WIDE_BATCH && (GNPDE_WIDE_NOFB || rows_fit_buffer<VEC, T>(off))) {
    const bool has_err = ERR && st.err_rows != nullptr;
    using WS = WideSlots<NOUT, NKMAX, ERR>;
    constexpr int N = WS::N;
    WS w;
    wide_slots<NOUT, NKMAX, ERR>(st, xid, w);
    const uint32_t bo = (uint32_t)(off * (int64_t)sizeof(T));
    // every operand row issued before any is used (one memory round trip); the first PK
    // present ones were read before the gathers (epi_prefetch, GNPDE_STG4_PRE)
    Packed<VEC, T> v[N];
    int cnt = 0;
#pragma unroll
    for (int q = 0; q < N; ++q) {
      bool from_pre = false;
      if constexpr (PK > 0) {
        if (pre && w.p[q]) {
#pragma unroll
          for (int c = 0; c < PK; ++c)
            if (cnt == c) {
              v[q] = pre[c];
              from_pre = true;
            }
        }
      }
      if (!from_pre) opt_load<VEC, T>(w.p[q], bo, v[q]);
      cnt += w.p[q] != nullptr;
    }
    const float* cb = w.cb;
#pragma unroll
    for (int q = 0; q < N; ++q) {
      const int slot = WS::slot(q);
      const Packed<VEC, T> vq = v[q];
      if (slot < NOUT) {
        const bool isx = xid != nullptr && slot < st.n_out && st.o[slot].base == xid;
#pragma unroll
        for (int t = 0; t < VEC; ++t) r[slot][t] = cb[slot] * (isx ? xv[t] : unpack(vq, t));
        if constexpr (DENSE) {
          if (slot == 0) {
            const bool on = st.n_out > 0 && st.o[0].base != nullptr;
#pragma unroll
            for (int t = 0; t < VEC; ++t) rd[t] = on ? dc[0] * (isx ? xv[t] : unpack(vq, t)) : 0.f;
          }
        }
        if (ERR && y0v && has_err && w.p[q] != nullptr && w.p[q] == st.err_y0) *y0v = vq;  // y0 = this base
      } else if (slot < NOUT + NKMAX) {
        const int j = slot - NOUT;
        const bool on = j < st.nk;
        const bool kx = on && xid != nullptr && st.k[j] == xid;  // the RHS input row, already held
        float kv[VEC];
#pragma unroll
        for (int t = 0; t < VEC; ++t) kv[t] = kx ? xv[t] : unpack(vq, t);
#pragma unroll
        for (int i = 0; i < NOUT; ++i) {
          const float c = (on && i < st.n_out) ? st.o[i].c[j] * sco[i] : 0.f;
#pragma unroll
          for (int t = 0; t < VEC; ++t) r[i][t] = fmaf(c, kv[t], r[i][t]);
        }
        if constexpr (DENSE) {
          const float c = on ? dc[1 + j] : 0.f;
#pragma unroll
          for (int t = 0; t < VEC; ++t) rd[t] = fmaf(c, kv[t], rd[t]);
        }
        if constexpr (ERR) {
          const float c = (on && has_err) ? st.err.c[j] * sc : 0.f;
#pragma unroll
          for (int t = 0; t < VEC; ++t) ev[t] = fmaf(c, kv[t], ev[t]);
        }
      } else if (slot == NOUT + NKMAX) {
        if constexpr (ERR) {
          const bool isx = xid != nullptr && has_err && st.err.base == xid;
#pragma unroll
          for (int t = 0; t < VEC; ++t) ev[t] = cb[NOUT] * (isx ? xv[t] : unpack(vq, t));
        }
      } else if (y0v) {  // the tolerance's y0
        if (w.p[q] != nullptr)
          *y0v = vq;
        else if (ERR && has_err && xid != nullptr && st.err_y0 == xid)  // the RHS input row, held
          pack_into<VEC, T>(xv, *y0v);
        // (otherwise NULL: deduplicated against a base, copied above)
      }
    }
#pragma unroll
    for (int i = 0; i < NOUT; ++i) {
      const float cf = i < st.n_out ? st.o[i].cf * sco[i] : 0.f;
#pragma unroll
      for (int t = 0; t < VEC; ++t) r[i][t] = fmaf(cf, o[t], r[i][t]);
    }
    if constexpr (ERR) {
      const float cf = has_err ? st.err.cf * sc : 0.f;
#pragma unroll
      for (int t = 0; t < VEC; ++t) ev[t] = fmaf(cf, o[t], ev[t]);
    }
    if constexpr (DENSE) {
#pragma unroll
      for (int t = 0; t < VEC; ++t) rd[t] = fmaf(dc[kDenseSlots - 1], o[t], rd[t]);
    }
    return;
  }
  // (the fallback for rows past the buffer range: an operand equal to the RHS input is
  // loaded like any other and its value replaced by the held row — a branch between the
  // held row and a load is folded into a load through a selected pointer, which puts xv
  // in scratch memory for every row of the kernel)
  auto base_term = [&](const gnpde_stage_out_t& so, float (&acc)[VEC]) {
    if (so.base == nullptr) {
#pragma unroll
      for (int t = 0; t < VEC; ++t) acc[t] = 0.f;
    } else {
      const bool isx = xid != nullptr && so.base == xid;
      Packed<VEC, T> bv;
      load_packed<VEC>(as_t<T>(so.base) + off, bv);
#pragma unroll
      for (int t = 0; t < VEC; ++t) acc[t] = so.cb * (isx ? xv[t] : unpack(bv, t));
    }
  };
  const bool has_err = ERR && st.err_rows != nullptr;
  if (y0v && has_err) load_packed<VEC>(as_t<T>(st.err_y0) + off, *y0v);  // err_terms reads it from y0v
#pragma unroll
  for (int i = 0; i < NOUT; ++i)
    if (i < st.n_out) base_term(st.o[i], r[i]);
  if (has_err) base_term(st.err, ev);
  if constexpr (DENSE) {
    if (st.n_out > 0) {
      gnpde_stage_out_t so = st.o[0];
      so.cb = dc[0];
      base_term(so, *reinterpret_cast<float(*)[VEC]>(rd));
    } else {
#pragma unroll
      for (int t = 0; t < VEC; ++t) rd[t] = 0.f;
    }
  }
#pragma unroll
  for (int j = 0; j < NKMAX; ++j) {
    if (j < st.nk) {
      const bool kx = xid != nullptr && st.k[j] == xid;
      Packed<VEC, T> kp;
      load_packed<VEC>(as_t<T>(st.k[j]) + off, kp);
      float kv[VEC];
#pragma unroll
      for (int t = 0; t < VEC; ++t) kv[t] = kx ? xv[t] : unpack(kp, t);
#pragma unroll
      for (int i = 0; i < NOUT; ++i) {
        if (i < st.n_out) {
          const float c = st.o[i].c[j] * sco[i];
#pragma unroll
          for (int t = 0; t < VEC; ++t) r[i][t] = fmaf(c, kv[t], r[i][t]);
        }
      }
      if (has_err) {
        const float c = st.err.c[j] * sc;
#pragma unroll
        for (int t = 0; t < VEC; ++t) ev[t] = fmaf(c, kv[t], ev[t]);
      }
      if constexpr (DENSE) {
#pragma unroll
        for (int t = 0; t < VEC; ++t) rd[t] = fmaf(dc[1 + j], kv[t], rd[t]);
      }
    }
  }
#pragma unroll
  for (int i = 0; i < NOUT; ++i) {
    if (i < st.n_out) {
      const float cf = st.o[i].cf * sco[i];
#pragma unroll
      for (int t = 0; t < VEC; ++t) r[i][t] = fmaf(cf, o[t], r[i][t]);
    }
  }
  if (has_err) {
    const float cf = st.err.cf * sc;
#pragma unroll
    for (int t = 0; t < VEC; ++t) ev[t] = fmaf(cf, o[t], ev[t]);
  }
  if constexpr (DENSE) {
#pragma unroll
    for (int t = 0; t < VEC; ++t) rd[t] = fmaf(dc[kDenseSlots - 1], o[t], rd[t]);
  }
}

// sum_t (e_t / tol_t)^2 with tol = atol + rtol * max(|y0|, |y1|): the slice's share of
// the embedded pair's squared error norm.  tol and the quotient in fp32 as torchdiffeq
// forms them on an fp32 state (_compute_error_ratio: the 0-d fp64 atol / rtol do not
// promote it), the squares summed in fp64 (round 6; the quotient was fp64, whose
// division sequence cost the f0 / probe launches of the initial step 40-50 us each).
// err_y1 = -2: tol = atol + rtol |y0| (y1 ignored).  aux (scale_rows): += sum (y0 / tol)^2.
template <int VEC, class T>
__device__ __forceinline__ double err_terms(const gnpde_stage_epilogue_t& st, int64_t off, const float (&ev)[VEC],
                                            const float (&y1)[VEC], const Packed<VEC, T>* y0pre = nullptr,
                                            double* aux = nullptr) {
  Packed<VEC, T> y0v;
  if (GNPDE_WIDE_BATCH && y0pre)  // loaded with the operands (wide_combine)
    y0v = *y0pre;
  else
    load_packed<VEC>(as_t<T>(st.err_y0) + off, y0v);
  if constexpr (GNPDE_ERR_DIAG & 1) return (double)ev[0] + (double)unpack(y0v, 0);
  const bool y0only = st.err_y1 == -2;
  const float at = (float)st.atol, rt = (float)st.rtol;
  float d = 0.f, a = 0.f;
#pragma unroll
  for (int t = 0; t < VEC; ++t) {
    const float y = unpack(y0v, t);
    const float ay0 = fabsf(y);
    const float tol = __fadd_rn(at, __fmul_rn(rt, y0only ? ay0 : fmaxf(ay0, fabsf(y1[t]))));  // no fma: torch rounds twice
    const float q = ev[t] / tol;
    d = fmaf(q, q, d);
    if (aux) {  // (the f0 launch of an adaptive solve only: tol is then atol + rtol |y0|)
      const float qy = y / tol;
      a = fmaf(qy, qy, a);
    }
  }
  if (aux) *aux += (double)a;
  return (double)d;
}

// f = a*(ax - x) [+ b*x0]  (function_laplacian_diffusion.py:69-77) or f = ax,
// then either store f or emit the fused Runge-Kutta stage outputs.  dpart
// accumulates the row's dot term (STG 2, 3) or error term (STG 4) of this slice;
// STG 4 takes dpart[2]: the error term in dpart[0], its dot term in dpart[1].
template <int VEC, int STG, class T = float>
__device__ __forceinline__ void epi_finish(const Epi& e, int64_t row, int cc, const float (&ax)[VEC], float a,
                                           float b, const EpiPre<VEC, T, STG>& p, double* dpart = nullptr) {
  float o[VEC];
  const bool need_x = (e.flags & GNPDE_EPI_RHS) != 0;
  if (need_x) {
#pragma unroll
    for (int t = 0; t < VEC; ++t) o[t] = a * (ax[t] - unpack(p.xr, t));
    if (e.flags & GNPDE_ADD_SOURCE) {
#pragma unroll
      for (int t = 0; t < VEC; ++t) o[t] = o[t] + b * unpack(p.x0r, t);
    }
  } else {
#pragma unroll
    for (int t = 0; t < VEC; ++t) o[t] = ax[t];
  }
  if constexpr (!STG) {
    store_vec<VEC>(as_t<T>(e.f) + row * e.ldf + cc, o);
    return;
  }
  if (e.st.f_lin != 0.f && need_x) {  // f = x + sc*f_lin*f: the affine stage derivative (ABI 5)
    const float cl = stage_scale(e.st) * e.st.f_lin;
#pragma unroll
    for (int t = 0; t < VEC; ++t) o[t] = fmaf(cl, o[t], unpack(p.xr, t));
  }
  const int64_t off = row * e.ldf + cc;
  if (e.st.f_out) store_vec<VEC>(as_t<T>(e.st.f_out) + off, o);
  // the stage outputs' row (out_rows: the last step of a renumbered solve writes the caller's numbering)
  const int64_t oo = e.st.out_rows ? (int64_t)e.st.out_rows[row] * e.ldf + cc : off;
  if constexpr (stage_wide<STG>()) {
    constexpr bool DENSE = STG == 5;
    float xv[VEC], r[2][VEC], ev[VEC], rd[VEC];
    Packed<VEC, T> y0v;
#pragma unroll
    for (int t = 0; t < VEC; ++t) xv[t] = need_x ? unpack(p.xr, t) : 0.f;
    DenseCoef dc;
    if constexpr (DENSE) dc = dense_load(e.st);
    wide_combine<VEC, T, GNPDE_STAGE_MAX_K, 2, true, GNPDE_STG4_PRE, DENSE>(
        e.st, off, o, (need_x && e.ldx == e.ldf) ? e.x : nullptr, xv, r, ev, &y0v, GNPDE_STG4_PRE > 0 ? p.wk : nullptr,
        DENSE ? dc.c : nullptr, DENSE ? rd : nullptr);
#pragma unroll
    for (int i = 0; i < 2; ++i)
      if (i < e.st.n_out) store_vec<VEC>(as_t<T>(e.st.o[i].out) + oo, r[i]);
    if constexpr (DENSE) {
      if (dc.on) {  // wave-uniform: the step crosses the output time
        T* dout = reinterpret_cast<T*>(*e.st.dense_out);
        const int64_t od = e.st.dense_rows ? (int64_t)e.st.dense_rows[row] * e.ldf + cc : off;
        store_vec<VEC>(dout + od, rd);
      }
    }
    if (e.st.err_rows && dpart) {
      float y1[VEC];
#pragma unroll
      for (int t = 0; t < VEC; ++t) y1[t] = e.st.err_y1 == 1 ? r[1][t] : (e.st.err_y1 == 0 ? r[0][t] : xv[t]);
      dpart[0] += err_terms<VEC, T>(e.st, off, ev, y1, &y0v, e.st.scale_rows ? &dpart[1] : nullptr);
    }
    // the dot term of the wide epilogue (its second row sum, dpart[1]): <f, dot_with> of the
    // row slice, f as the other epilogues take it (after f_lin)
    if constexpr (sizeof(T) == 4) {  // (fp32 state only: the bf16 K1 rejects dot terms)
      if (e.st.dot_rows && dpart) {
        Packed<VEC, T> dw;
        load_packed<VEC>(as_t<T>(e.st.dot_with) + off, dw);
#pragma unroll
        for (int t = 0; t < VEC; ++t) dpart[1] = fma((double)o[t], (double)unpack(dw, t), dpart[1]);
      }
    }
    return;
  } else {
    if constexpr (stage_dot<STG>()) {
      if (e.st.dot_rows && dpart) {
        Packed<VEC, T> dw;
        if constexpr (stage_dw_pre<STG>())
          dw = p.dw;
        else
          load_packed<VEC>(as_t<T>(e.st.dot_with) + off, dw);
        if constexpr (GNPDE_DOT_DIAG == 1) {
          *dpart += (double)unpack(dw, 0);
        } else {
#pragma unroll
          for (int t = 0; t < VEC; ++t) *dpart = fma((double)o[t], (double)unpack(dw, t), *dpart);
        }
      }
    }
    const float sc = stage_scale(e.st);
    if constexpr (!stage_prefetch<STG>()) {
      // no prefetch: the stage operands streamed after the gathers (wide_combine, the
      // same per-output order as stage_combine: same bits)
      constexpr int NO = stage_nout<STG>();
      float xv[VEC], r[2][VEC], ev[VEC];
#pragma unroll
      for (int t = 0; t < VEC; ++t) xv[t] = need_x ? unpack(p.xr, t) : 0.f;
      wide_combine<VEC, T, kStagePre, NO, false>(e.st, off, o, (need_x && e.ldx == e.ldf) ? e.x : nullptr, xv, r,
                                                 ev);
#pragma unroll
      for (int i = 0; i < NO; ++i)
        if (i < e.st.n_out) store_vec<VEC>(as_t<T>(e.st.o[i].out) + oo, r[i]);
    } else {
      // the shared stage operands, prefetched before the gathers
      constexpr int NK = stage_kpre<STG>();
      auto kval = [&](int j, int t) -> float {
        return (need_x && e.st.k[j] == e.x && e.ldx == e.ldf) ? unpack(p.xr, t) : unpack(p.kv[j], t);
      };
#pragma unroll
      for (int i = 0; i < stage_nout<STG>(); ++i) {
        if (i >= e.st.n_out) break;
        float r[VEC];
        stage_combine<VEC, NK, T>(e, e.st.o[i], off, o, p.xr, &p.base[i], kval, out_scale(e.st, i, sc), r);
        store_vec<VEC>(as_t<T>(e.st.o[i].out) + oo, r);
      }
    }
  }
}

template <int VEC, int STG, class T = float>
__device__ __forceinline__ void epilogue_store(const Epi& e, int64_t row, int cc, const float (&ax)[VEC], float a,
                                               float b, double* dpart = nullptr) {
  EpiPre<VEC, T, STG> p;
  epi_prefetch<VEC, STG, T>(e, row, cc, p);
  epi_finish<VEC, STG, T>(e, row, cc, ax, a, b, p, dpart);
}

// Whether an instantiation has a per-row fp64 term to reduce and store (the dot
// term of the adjoint stages on fp32 rows, the error rows of the wide epilogue).
template <int STG, class T>
constexpr bool stage_rowsum() {
  return (stage_dot<STG>() && sizeof(T) == 4) || stage_err<STG>();
}


// an fp64 value moved by DPP (each 32-bit half), bound controls as in flash.hip's dpp_mov
template <int CTRL>
__device__ __forceinline__ double dpp_mov64(double v) {
  const u32x2 w = __builtin_bit_cast(u32x2, v);
  const u32x2 r = {(uint32_t)__builtin_amdgcn_update_dpp(0, (int)w.x, CTRL, 0xf, 0xf, false),
                   (uint32_t)__builtin_amdgcn_update_dpp(0, (int)w.y, CTRL, 0xf, 0xf, false)};
  return __builtin_bit_cast(double, r);
}

// Sum over aligned groups of GL lanes (GL a power of two), every lane of a group
// ending with the group's sum: DPP inside 16-lane rows (xor 1, xor 2, then the
// half-row and row mirrors, which pair lanes holding equal partial sums), a
// cross-lane shuffle per further doubling.  A fixed order: deterministic.
// (An xor tree of 64-bit shuffles costs two LDS-unit permutes per step; the
// adjoint launch's row dot term measured 27 us of a 117-us launch that way.)
template <int GL>
__device__ __forceinline__ double group_sum64(double v) {
  if constexpr (GL >= 2) v += dpp_mov64<0xB1>(v);   // quad_perm [1,0,3,2]
  if constexpr (GL >= 4) v += dpp_mov64<0x4E>(v);   // quad_perm [2,3,0,1]
  if constexpr (GL >= 8) v += dpp_mov64<0x141>(v);  // row_half_mirror
  if constexpr (GL >= 16) v += dpp_mov64<0x140>(v); // row_mirror
#pragma unroll
  for (int o = 16; o < GL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// The same in fp32 (the error / scale rows of the wide epilogue: fp32 quotients whose
// squares torchdiffeq itself sums in fp32): one DPP add per step, one permute per
// further doubling — a shorter chain at the end of every wave than the fp64 tree.
template <int CTRL>
__device__ __forceinline__ float dpp_mov32(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xf, 0xf, false));
}

template <int GL>
__device__ __forceinline__ float group_sum32(float v) {
  if constexpr (GL >= 2) v += dpp_mov32<0xB1>(v);
  if constexpr (GL >= 4) v += dpp_mov32<0x4E>(v);
  if constexpr (GL >= 8) v += dpp_mov32<0x141>(v);
  if constexpr (GL >= 16) v += dpp_mov32<0x140>(v);
#pragma unroll
  for (int o = 16; o < GL; o <<= 1) v += __shfl_xor(v, o);
  return v;
}

// prev: the row's running dot read before the gathers (GNPDE_DOT_PRE), or nullptr;
// dot_ch: the dot channel whatever err_rows says (the wide epilogue's second row sum)
__device__ __forceinline__ void epi_rowsum_write(const Epi& e, int64_t row, double v, const double* prev = nullptr,
                                                 bool dot_ch = false) {
  if (dot_ch && e.st.scale_rows) {  // the wide epilogue's second row sum as scale_rows (ABI 8)
    e.st.scale_rows[row] = v;
  } else if (e.st.err_rows && !dot_ch) {
    e.st.err_rows[row] = v;
  } else if (e.st.dot_rows) {
    double* d = e.st.dot_rows + row;
    const double w = e.st.dot_coef * v;
    *d = e.st.dot_accumulate ? (prev ? *prev : *d) + w : w;
  }
}

// The row's dot / error term: the owner lanes' partials (lanes [base, base + GL)
// of the wavefront, GL a power of two, base a multiple of GL) summed by a fixed
// xor tree, stored by the first of them.  Called by every lane of the row's slot
// (convergent).
template <int GL, bool F32 = false>
__device__ __forceinline__ void epi_rowsum_store(const Epi& e, int64_t row, double dpart, bool store,
                                                 const double* prev = nullptr, bool dot_ch = false) {
  static_assert((GL & (GL - 1)) == 0, "the xor tree needs power-of-two row lanes");
  if constexpr (GNPDE_DOT_DIAG == 2) return;
  if constexpr (F32)
    dpart = (double)group_sum32<GL>((float)dpart);
  else
    dpart = group_sum64<GL>(dpart);
  if (store) epi_rowsum_write(e, row, dpart, prev, dot_ch);
}

// The same for any GL (e.g. 21 lanes: three bf16 rows of 168 columns per wavefront):
// the first owner lane sums the slot's lanes base .. base + GL - 1 in order.
template <int GL, bool F32 = false>
__device__ __forceinline__ void epi_rowsum_store_any(const Epi& e, int64_t row, double dpart, int base, bool store,
                                                     const double* prev = nullptr, bool dot_ch = false) {
  if constexpr ((GL & (GL - 1)) == 0) {
    epi_rowsum_store<GL, F32>(e, row, dpart, store, prev, dot_ch);
  } else {
    double tot = 0.0;
#pragma unroll
    for (int j = 0; j < GL; ++j) tot += __shfl(dpart, base + j);
    if (store) epi_rowsum_write(e, row, tot, prev, dot_ch);
  }
}

// The row sums of an epilogue (wave-uniform branches; called by every lane of the
// row's slot): STG 2 / 3 the dot term (dpart[0]); STG 4 the error rows (dpart[0])
// and the dot term (dpart[1]).
template <int GL, int STG, class T>
__device__ __forceinline__ void epi_rowsums(const Epi& e, int64_t row, const double* dpart, int base, bool store,
                                            const double* prev = nullptr) {
  if constexpr (stage_rowsum<STG, T>()) {
    if constexpr (stage_wide<STG>()) {
      if constexpr (GNPDE_ERR_DIAG & 2) return;
      // the error / scale rows: fp32 slice sums (err_terms), reduced in fp32 and stored as fp64
      if (e.st.err_rows) epi_rowsum_store_any<GL, true>(e, row, dpart[0], base, store);
      if (e.st.scale_rows) {
        epi_rowsum_store_any<GL, true>(e, row, dpart[1], base, store, nullptr, true);
      } else if constexpr (sizeof(T) == 4) {
        if (e.st.dot_rows) epi_rowsum_store_any<GL>(e, row, dpart[1], base, store, nullptr, true);
      }
    } else {
      if (e.st.dot_rows || e.st.err_rows) epi_rowsum_store_any<GL>(e, row, dpart[0], base, store, prev);
    }
  }
}

inline int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// The STG instantiation an epilogue needs: 0 = store f, 1 = one stage output
// and no dot term (the forward Runge-Kutta steps), 3 = one stage output and the
// dot term (three of the four adjoint launches of an rk4 step), 2 = the general
// epilogue, 4 = the wide epilogue (error rows or more than kStagePre operands:
// the adaptive solvers).
inline int epi_stage_kind(const Epi& e) {
  if (!e.has_stage) return 0;
  if (e.st.err_rows || e.st.nk > kStagePre || e.st.dense_out) return 4;  // (5 = 4 + dense_out: launch_agg_cfg)
  if (e.st.n_out <= 1) return e.st.dot_rows ? 3 : 1;
  return 2;
}

// Write-through (sc1) stores of VEC floats at byte offset off: the bytes reach
// the memory side before the storing wave's s_waitcnt vmcnt(0) returns, so a
// workgroup on any XCD can read them after an agent-scope acquire (the in-launch
// hand-off of cdna_hip_programming.md §6 Guideline 16, R1) with no release fence.
constexpr int kAuxSc1 = 16;

template <int VEC>
__device__ __forceinline__ void buf_store_wt(__amdgpu_buffer_rsrc_t r, uint32_t off, const float (&v)[VEC]) {
  if constexpr (VEC >= 4) {
#pragma unroll
    for (int q = 0; q < VEC / 4; ++q) {
      const u32x4 d = {__builtin_bit_cast(uint32_t, v[4 * q]), __builtin_bit_cast(uint32_t, v[4 * q + 1]),
                       __builtin_bit_cast(uint32_t, v[4 * q + 2]), __builtin_bit_cast(uint32_t, v[4 * q + 3])};
      // a dropped store (kBufNone) stays dropped: kBufNone + 16 would wrap to offset 0
      const uint32_t o = off >= kBufRecords ? kBufNone : off + 16u * q;
      __builtin_amdgcn_raw_buffer_store_b128(d, r, o, 0, kAuxSc1);
    }
  } else if constexpr (VEC == 2) {
    const u32x2 d = {__builtin_bit_cast(uint32_t, v[0]), __builtin_bit_cast(uint32_t, v[1])};
    __builtin_amdgcn_raw_buffer_store_b64(d, r, off, 0, kAuxSc1);
  } else {
    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, v[0]), r, off, 0, kAuxSc1);
  }
}

// write-through store of one double (as buf_store_wt)
__device__ __forceinline__ void buf_store_wt_f64(__amdgpu_buffer_rsrc_t r, uint32_t off, double v) {
  __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u32x2, v), r, off, 0, kAuxSc1);
}

}  // namespace gnpde
