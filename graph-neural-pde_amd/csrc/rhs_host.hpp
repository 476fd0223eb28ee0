// rhs_host.hpp — host-side argument checks and packing shared by the RHS
// translation units (rhs.hip: K1 and the unfused attention pieces;
// attention.hip: the fused attention RHS).
#pragma once
#include <cstdlib>

#include "scores.hpp"

namespace gnpde {

inline int check_score_args(int mode, int64_t heads, int64_t dk, const double* cs, const float* q, const float* k) {
  GNPDE_REQUIRE(heads >= 1 && heads <= 16, GNPDE_EUNSUPPORTED, "attention: heads=%lld not in [1,16]",
                (long long)heads);
  GNPDE_REQUIRE(mode >= GNPDE_SCORE_REFERENCE && mode <= GNPDE_SCORE_UNIFORM, GNPDE_EINVAL,
                "attention: unknown score mode %d", mode);
  if (mode == GNPDE_SCORE_REFERENCE) {
    GNPDE_REQUIRE(cs != nullptr, GNPDE_EINVAL, "attention: reference mode needs cs");
  } else if (mode != GNPDE_SCORE_UNIFORM) {
    GNPDE_REQUIRE(q != nullptr && k != nullptr && dk >= 1, GNPDE_EINVAL, "attention: per-edge mode needs q, k, dk");
  }
  return GNPDE_OK;
}

inline ScoreArgs make_score_args(int mode, int64_t heads, int64_t dk, const double* cs, const float* q,
                                 const float* k, int64_t ldqk, float p0, float p1) {
  ScoreArgs sa;
  sa.mode = mode;
  sa.H = (int)heads;
  sa.dk = (int)dk;
  sa.cs = cs;
  sa.q = q;
  sa.k = k;
  sa.ldqk = ldqk;
  sa.p0 = p0;
  sa.p1 = p1;
  return sa;
}

// Experiment knob (not part of the ABI contract): GNPDE_XCD_REMAP=1 maps
// contiguous eighths of the K1 work items to one XCD each; =K (>= 2) deals
// chunks of K consecutive blocks to the XCDs in turn (common.hpp xcd_block).
inline int xcd_remap_enabled() {
  if constexpr (!GNPDE_EXPERIMENTS) return 0;
  static const int on = [] {
    const char* e = std::getenv("GNPDE_XCD_REMAP");
    return e ? std::max(0, std::atoi(e)) : 0;
  }();
  return on;
}

// The stage struct's own consistency (include/gnpde.h, fused solver epilogue).
inline int check_stage(const gnpde_stage_epilogue_t& st) {
  GNPDE_REQUIRE(st.n_out >= 0 && st.n_out <= GNPDE_STAGE_MAX_OUT, GNPDE_EINVAL, "stage: n_out out of range");
  GNPDE_REQUIRE(st.nk >= 0 && st.nk <= GNPDE_STAGE_MAX_K, GNPDE_EINVAL, "stage: nk=%d out of [0, %d]", st.nk,
                GNPDE_STAGE_MAX_K);
  for (int j = 0; j < st.nk; ++j) GNPDE_REQUIRE(st.k[j] != nullptr, GNPDE_EINVAL, "stage: k[%d] is NULL", j);
  for (int i = 0; i < st.n_out; ++i) GNPDE_REQUIRE(st.o[i].out, GNPDE_EINVAL, "stage: output %d is NULL", i);
  GNPDE_REQUIRE(st.f_out || st.n_out > 0 || st.err_rows, GNPDE_EINVAL, "stage: the epilogue stores nothing");
  GNPDE_REQUIRE(!st.dot_rows || st.dot_with, GNPDE_EINVAL, "stage: dot_rows without dot_with");
  // a dot term beside error rows or more than kStagePre operands: the wide epilogue (STG 4)
  // carries it as a second row sum (the adaptive adjoint's alpha integrand, gnpde.integrator)
  if (st.err_rows) {
    GNPDE_REQUIRE(st.err_y0 != nullptr, GNPDE_EINVAL, "stage: err_rows without err_y0");
    GNPDE_REQUIRE(st.err_y1 >= -2 && st.err_y1 < st.n_out, GNPDE_EINVAL, "stage: err_y1=%d names no output",
                  st.err_y1);
    GNPDE_REQUIRE(st.atol >= 0.0 && st.rtol >= 0.0 && (st.atol > 0.0 || st.rtol > 0.0), GNPDE_EINVAL,
                  "stage: tolerances must be >= 0 and not both 0");
  }
  // the folded dense output (ABI 8): its device slot and coefficient table; the launch
  // that forms the table: its times and step size
  if (st.dense_out) GNPDE_REQUIRE(st.dense_tab, GNPDE_EINVAL, "stage: dense_out without dense_tab");
  if (st.dense_tab && !st.dense_out)
    GNPDE_REQUIRE(st.dense_t && st.dense_dt, GNPDE_EINVAL, "stage: dense_tab without dense_t / dense_dt");
  GNPDE_REQUIRE(!st.scale_rows || (st.err_rows && !st.dot_rows), GNPDE_EINVAL,
                "stage: scale_rows needs err_rows and no dot_rows");
  return GNPDE_OK;
}

inline Epi make_epi(const float* x, int64_t ldx, const float* x0, int64_t ldx0, const float* alpha, const float* beta,
                    int flags, float* f, int64_t ldf, const gnpde_stage_epilogue_t* stage = nullptr) {
  Epi e{};
  e.xcd_remap = xcd_remap_enabled();
  e.has_stage = stage != nullptr;
  if (stage) e.st = *stage;
  e.x = x;
  e.ldx = ldx;
  e.x0 = x0;
  e.ldx0 = ldx0;
  e.alpha = alpha;
  e.beta = beta;
  e.flags = flags;
  e.f = f;
  e.ldf = ldf;
  return e;
}

inline int check_epi(const Epi& e, int64_t C, int64_t n_heavy, const void* partials, int64_t n_slots) {
  GNPDE_REQUIRE(C >= 1, GNPDE_EINVAL, "rhs: C must be >= 1");
  GNPDE_REQUIRE(e.x && (e.f || e.has_stage), GNPDE_EINVAL, "rhs: NULL x or f");
  if (e.has_stage) {
    int rc = check_stage(e.st);
    if (rc) return rc;
  }
  GNPDE_REQUIRE(e.ldx >= C && e.ldf >= C, GNPDE_EINVAL, "rhs: leading dimension < C");
  if (e.flags & GNPDE_EPI_RHS) GNPDE_REQUIRE(e.alpha != nullptr, GNPDE_EINVAL, "rhs: NULL alpha");
  if (e.flags & GNPDE_ADD_SOURCE) {
    GNPDE_REQUIRE(e.flags & GNPDE_EPI_RHS, GNPDE_EINVAL, "rhs: ADD_SOURCE needs EPI_RHS");
    GNPDE_REQUIRE(e.x0 && e.beta && e.ldx0 >= C, GNPDE_EINVAL, "rhs: ADD_SOURCE needs x0, beta, ldx0 >= C");
  }
  GNPDE_REQUIRE(n_heavy == 0 || (partials != nullptr && n_slots > 0), GNPDE_EINVAL,
                "rhs: hub rows need a partials buffer and its slot count");
  // hub partials are addressed with 32-bit buffer offsets (aggregate.hpp, buf_store_wt)
  GNPDE_REQUIRE(n_slots >= 0 && (n_heavy == 0 || n_slots * C * 4 < (int64_t)kBufRecords), GNPDE_EUNSUPPORTED,
                "rhs: %lld hub partial slots x %lld columns exceed the 4 GiB of 32-bit buffer offsets; plan the "
                "graph with a larger chunk", (long long)n_slots, (long long)C);
  return GNPDE_OK;
}

// team geometry for the per-edge modes: VEC = 4, S = dk/4, T = H*S, both powers
// of two, T <= 64; otherwise lane mode (T = 0).
inline bool team_mode_enabled() {  // GNPDE_TEAM=0 forces lane mode (diagnostics)
  static const bool on = [] {
    const char* e = std::getenv("GNPDE_TEAM");
    return !(e && e[0] == '0');
  }();
  return on;
}

inline Team team_geometry(const ScoreArgs& sa) {
  Team tm{0, 0};
  if (!team_mode_enabled()) return tm;
  if (sa.mode != GNPDE_SCORE_DOT && sa.mode != GNPDE_SCORE_EXP_KERNEL && sa.mode != GNPDE_SCORE_COSINE &&
      sa.mode != GNPDE_SCORE_PEARSON)
    return tm;
  if (sa.dk % 4 != 0 || sa.ldqk % 4 != 0 || !aligned16(sa.q) || !aligned16(sa.k)) return tm;
  const int S = sa.dk / 4, T = sa.H * S;
  if ((S & (S - 1)) || (T & (T - 1)) || T > kWave) return tm;
  tm.T = T;
  tm.S = S;
  return tm;
}

}  // namespace gnpde
