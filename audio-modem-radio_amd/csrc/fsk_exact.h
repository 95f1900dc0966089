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
  double* rows;            // [B][2][m] the flagged streams' filtfilt rows (the plan's z), by ordinal
  double* slots;           // [n_slots][slot_doubles] envelope scratch (E2)
  int64_t slot_doubles;
  int n_slots;
  const PfLen* L;          // pocketfft's plans of length n (device copy)
  const double* pool;
  double fct;              // double(1 / long double n)
  uint8_t* xbits;          // [B][bits_stride] exact compare bits, F3 reads them for flagged streams
};

// the flagged streams of the batch (x: B rows, x_stride apart) -> their exact
// compare bits in X.xbits; every kernel exits at once when nothing is flagged
hipError_t launch_fsk_exact(int dtype, const void* x, int64_t x_stride, int64_t B, const FskParams& p,
                            const FskIir& f, const FskExact& X, hipStream_t st);

}  // namespace amr
