// dn_internal.hpp — shared declarations of the native library (not part of the C-ABI).
#pragma once

#include <cstdint>
#include <cstdlib>

#include "dn_shamir.h"

namespace dn {
// A/B tuning knobs (grid cap, wave schedule, store policy, kernel variants).
// The product library is built without DN_TUNING: every knob reads as unset
// and the library consults no environment variable.  `make tuning` builds
// lib/libdn_shamir_tuning.so with -DDN_TUNING, where a knob is the DN_* env
// var of that name, read per call (scripts/ probes and variant tests only).
inline const char* tune_env(const char* name) {
#ifdef DN_TUNING
  return std::getenv(name);
#else
  (void)name;
  return nullptr;
#endif
}

// Record a thread-local error message and return `code` (printf-style).
int set_error(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

// Forward differences (split by additions) stay below 2^544 while
// sum_{j<t} (n+t)^j < 2^23 (every table entry and every intermediate Newton
// coefficient is bounded by f at some x <= n + t - 1); otherwise the split
// folds after every Horner step.
inline bool fd_needs_fold(int t, int n) {
  double s = 0.0, p = 1.0;
  for (int j = 0; j < t; ++j) {
    s += p;
    p *= static_cast<double>(n + t);
  }
  return s >= 8388608.0;
}

// Compute units of the current device (cached per device; shamir_m521.hip).
int device_cu_count();

// MT19937 jump-ahead (host_mt_jump.cpp): substream length in words, the most
// substreams the jump table covers, a window stepped forward on the host, and
// CPython's final state after `words` outputs (false: beyond the table).
uint64_t mt_jump_words();
uint64_t mt_jump_max_subs();
void mt_advance_window(const uint32_t* win, uint64_t steps, uint32_t* out);
bool mt_final_state(const uint32_t* state, int idx, uint64_t words, uint32_t* fin, int32_t* fidx);

// Runtime direct jump rows (host_gf2poly.cpp): D_s = x^(L - 624 + (s - 1) L)
// mod P, L = 17 * 2^14 words, row s - 1 of kMtPolyWords uint64, for the
// windows a backward-generating draw of S <= kMtRtRows + 1 substreams needs
// (odd s < S and S - 1); computed on first use and cached; *version changes
// whenever rows were added (nullptr: no carry-less multiply on this host, or
// a row disagreed with the tabulated ones).
constexpr uint64_t kMtRtRows = 2048;
const uint64_t* mt_direct_rows_l14(uint64_t S, uint64_t* version);
// D_1 .. D_nrows in sequence into out[nrows][kMtPolyWords] (the build's
// generator of the embedded table, csrc/gen_mt_rt_rows.cpp); false: no
// carry-less multiply, or a row disagreed with the tabulated ones.
bool mt_rt_rows_compute(uint64_t* out, uint64_t nrows);
// out[kMtPolyWords] = x^e mod P (the jump polynomial of e words); false: no
// carry-less multiply on this host
bool mt_xpow_mod(uint64_t e, uint64_t* out);
// The generator's checksum of the embedded table (two words written after it).
void mt_rt_rows_checksum(const uint64_t* words, uint64_t n, uint64_t out[2]);
}  // namespace dn
