// pocketfft.h -- plans of the device restatement of pocketfft, the FFT library
// scipy.fft runs (scipy 1.15.3's bundled pocketfft C++ header), for the two
// reference steps whose results depend on its exact rounding:
//   |scipy.signal.hilbert(f)|      modem.fsk_demodulate (modem.py:309, 315):
//                                  the FSK exact path (fsk_exact_kernels.hip)
//   scipy.signal.resample(x, num)  decoder.decode_wav_file (decoder.py:385-387)
// The algorithm is the one oracle/amr_pocketfft.c restates and pins bit for bit
// against scipy on every length 1..2000 (tests/test_oracle_golden.py); the
// plans here are built on the host by the same rules (pocketfft_plan.cpp) and
// executed by pocketfft_dev.h, one workgroup per transform.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace amr {

constexpr int kPfMaxF = 32;   // factors of one plan (a length < 2^31 has at most 30)

// one factor of a plan: radix ip, l1 = product of the factors before it,
// ido = len / (l1 * ip); tw / tws: offsets (in doubles) of its twiddles and of
// the generic passes' extra table in the plan's pool, -1 when absent
struct PfFact {
  int64_t ip, l1, ido, tw, tws;
};

// an FFTPACK-style plan (pocketfft's cfftp or rfftp)
struct PfPasses {
  int64_t len;
  int nf;
  PfFact f[kPfMaxF];
};

// pocketfft's fftblue(n): chirp bk (n complex), FFT of the padded chirp / n2
// bkf (n2 / 2 + 1 complex), a cfftp plan of n2 = good_size(2n - 1)
struct PfBlue {
  int64_t n, n2;
  int64_t bk, bkf;
  PfPasses plan;
};

// pocketfft_r(n) and pocketfft_c(n): rblue / cblue pick Bluestein (shared
// fftblue), else the rfftp plan r / cfftp plan c
struct PfLen {
  int64_t n;
  int rblue, cblue;
  PfPasses r, c;
  PfBlue bl;
};

// host: the plans of length n, twiddles appended to pool (aligned to a
// complex); bkf (Bluestein) is left to pf_finish on the device
bool pf_len_build(int64_t n, PfLen& L, std::vector<double>& pool);
// doubles of per-transform scratch pf_hilbert_env / pf_r2hc / pf_hc2r need
// beside the row itself (pocketfft_dev.h PfScratch); the same from n alone
int64_t pf_scratch_doubles(const PfLen& L);
int64_t pf_scratch_doubles_n(int64_t n);
// an upper bound on the pool pf_len_build(n) fills (host arithmetic only)
int64_t pf_pool_doubles_bound(int64_t n);
// device: fills bkf of every Bluestein plan in dL (L: the host copy), using
// tmp (>= 4 * n2 doubles of device scratch); synchronous on st
hipError_t pf_finish(const PfLen& L, const PfLen* dL, double* dpool, double* tmp, hipStream_t st);

// scipy.signal.resample(x, num) of `batch` real rows (decoder.py:385-387) on
// the device, bit for bit: Lx / Ly plans of nx / num (device copies), slots:
// per-workgroup scratch of resample_slot_doubles each
int64_t pf_resample_slot_doubles(const PfLen& Lx, const PfLen& Ly);
hipError_t launch_pf_resample(const PfLen* dLx, const double* poolx, const PfLen* dLy, const double* pooly,
                              const double* x, int64_t nx, double* y, int64_t num, int64_t batch, double* slots,
                              int64_t slot_doubles, int n_slots, double fct, double scale, hipStream_t st);

// |scipy.signal.hilbert(x)| of `batch` real rows of x, in place (diagnostic
// entry amr_hilbert_env_exact_host; the FSK exact path runs the same routine)
hipError_t launch_pf_hilbert_env(const PfLen* dL, const double* pool, double* x, int64_t n, int64_t batch,
                                 double* slots, int64_t slot_doubles, int n_slots, double fct, hipStream_t st);

}  // namespace amr
