// fsk_exact.h -- the FSK path's exact recomputation of streams whose compare
// bits the fast path cannot guarantee (fsk_exact_kernels.hip, DESIGN.md §2
// item 6).  fsk_api.cpp owns the buffers.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "amr_internal.h"
#include "pocketfft.h"

namespace amr {


struct FskExact {
  const uint32_t* flags;   // [B / 32] F2's flags: bit s of word s / 32
  int32_t* list;           // [B] ordinal -> stream (E0)
  int32_t* count;          // [1] flagged streams (E0)
  double* rows;            // the plan's z: (f_mark, f_space), then (env_mark, env_space) (see live)
  double* slots;           // [n_slots][slot_doubles] envelope scratch (E2)
  int64_t slot_doubles;
  int n_slots;
  const PfLen* L;          // pocketfft's plans of length n (device copy)
  const double* pool;
  double fct;              // double(1 / long double n)
  uint8_t* xbits;          // [B][bits_stride] exact compare bits, F3 reads them for flagged streams
  int fuse;                // LDS-fused transforms (pf_fuse_on)
  int lean;                // ... and every radix hard-coded: k_exact_env_lean
  int live_only;           // E2b stores only the live samples' envelopes (AMR_FSK_LIVEONLY=0: every sample, A/B)
  int xcd_pair;            // E2 rows of one stream on one XCD (AMR_FSK_XCDPAIR=0: off, A/B)
  // E2's grid: the persistent loops are correct at any size, so it is sized
  // from the counts the plan's last 8 launches saw (count_hint = their
  // maximum; E3 writes each to count_host, host-mapped) -- a few workgroups
  // after a run of clean batches, which then dispatch and exit without
  // waiting for room beside the other launches in flight; the full resident
  // grid while flagged batches keep coming
  int32_t* count_host;     // device pointer of a host-mapped int, or nullptr
  int64_t count_hint;
  // live (the plan's keep_z): rows is z itself, stream-indexed in the [L | D]
  // layout lc, whole after F2 -- no F1 re-run; the envelopes go back into z's
  // live samples, E3 reads them there.  Otherwise rows holds the F1 re-run's
  // output by ordinal, natural layout.
  int live;
  LiveCols lc;
};

// E0: F2's flags -> X.list / X.count.  Then F1 in list mode (fsk_api.cpp),
// then E2 + E3: the flagged streams' exact compare bits in X.xbits.  Every
// kernel exits at once when nothing is flagged.
hipError_t launch_fsk_exact_list(int64_t B, const FskExact& X, hipStream_t st);
hipError_t launch_fsk_exact_env(int64_t B, const FskParams& p, const FskExact& X, hipStream_t st,
                                bool env = true);

}  // namespace amr
