// fsk_exact.h -- the FSK exact fallback's transform plan (fsk_exact_kernels.hip,
// built on the host by fsk_api.cpp): pocketfft's factorisations of n and its
// twiddle tables, as oracle/amr_hilbert.c restates them.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "amr_internal.h"

namespace amr {

constexpr int kExactMaxFactors = 24;

struct ExactFft {
  int64_t n;
  int nr, nc;                          // real (rfftp) / complex (cfftp) factor counts
  int fr[kExactMaxFactors], fc[kExactMaxFactors];
  int64_t rto[kExactMaxFactors];       // offsets of each real factor's twiddles in rtw (doubles)
  int64_t cto[kExactMaxFactors];       // offsets of each complex factor's twiddles in ctw (complex)
  double fct;                          // double(1 / long double n)
  const double* rtw;
  const double2* ctw;
};

// the flagged streams of [s0, s0 + nb) (flags: that launch's words, s0 a
// multiple of 32; x: its rows) -> their exact compare bits in xbits (the
// batch's), which F3 reads
hipError_t launch_fsk_exact(int dtype, const void* x, int64_t x_stride, int64_t s0, int64_t nb, const uint32_t* flags,
                            int group, double* slots, int64_t slot_doubles, int n_slots, uint8_t* xbits, const FskParams& p,
                            const FskIir& f, const ExactFft& X, hipStream_t st);

}  // namespace amr
