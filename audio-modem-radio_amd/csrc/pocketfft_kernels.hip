// pocketfft_kernels.hip -- kernels over the device pocketfft restatement
// (pocketfft_dev.h): the Bluestein plans' bkf table (plan construction) and
// scipy.signal.resample for decode_wav_file (decoder.py:385-387), bit for bit.
//
// Derived from pocketfft (the FFT library bundled with scipy 1.15.3 as
// scipy.fft's pypocketfft), whose notice follows; the FFTPACK algorithms it
// implements are by Paul N. Swarztrauber (public domain).
//
//   Copyright (C) 2010-2019 Max-Planck-Society
//   All rights reserved.
//
//   Redistribution and use in source and binary forms, with or without
//   modification, are permitted provided that the following conditions are met:
//
//   * Redistributions of source code must retain the above copyright notice,
//     this list of conditions and the following disclaimer.
//   * Redistributions in binary form must reproduce the above copyright notice,
//     this list of conditions and the following disclaimer in the documentation
//     and/or other materials provided with the distribution.
//   * Neither the name of the copyright holder nor the names of its contributors
//     may be used to endorse or promote products derived from this software
//     without specific prior written permission.
//
//   THIS SOFTWARE IS PROVIDED BY THE COPYRIGHT HOLDERS AND CONTRIBUTORS "AS IS"
//   AND ANY EXPRESS OR IMPLIED WARRANTIES, INCLUDING, BUT NOT LIMITED TO, THE
//   IMPLIED WARRANTIES OF MERCHANTABILITY AND FITNESS FOR A PARTICULAR PURPOSE ARE
//   DISCLAIMED. IN NO EVENT SHALL THE COPYRIGHT HOLDER OR CONTRIBUTORS BE LIABLE
//   FOR ANY DIRECT, INDIRECT, INCIDENTAL, SPECIAL, EXEMPLARY, OR CONSEQUENTIAL
//   DAMAGES (INCLUDING, BUT NOT LIMITED TO, PROCUREMENT OF SUBSTITUTE GOODS OR
//   SERVICES; LOSS OF USE, DATA, OR PROFITS; OR BUSINESS INTERRUPTION) HOWEVER
//   CAUSED AND ON ANY THEORY OF LIABILITY, WHETHER IN CONTRACT, STRICT LIABILITY,
//   OR TORT (INCLUDING NEGLIGENCE OR OTHERWISE) ARISING IN ANY WAY OUT OF THE USE
//   OF THIS SOFTWARE, EVEN IF ADVISED OF THE POSSIBILITY OF SUCH DAMAGE.
#include <algorithm>
#include <cstdlib>

#include "amr_internal.h"
#include "pocketfft.h"
#include "pocketfft_dev.h"

namespace amr {

constexpr int kPfThreads = 512;

// fftblue's constructor: tbkf = bk / n2 zero-padded and mirrored, its
// forward cfftp transform, first n2 / 2 + 1 entries -> bkf (one workgroup)
__global__ __launch_bounds__(kPfThreads) void k_pf_bkf(const PfLen* __restrict__ L, double* pool, double* tmp,
                                                       int fuse) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  const PfBlue& B = L->bl;
  const int64_t n = B.n, n2 = B.n2;
  pf::Cx* tb = reinterpret_cast<pf::Cx*>(tmp);
  pf::Cx* ch = tb + n2;
  const pf::Cx* bk = reinterpret_cast<const pf::Cx*>(pool + B.bk);
  const double xn2 = 1.0 / (double)n2;
  for (int64_t m = threadIdx.x; m < n2; m += blockDim.x) {
    pf::Cx v = {0., 0.};
    if (m < n) v = pf::scale(bk[m], xn2);
    else if (m > n2 - n) v = pf::scale(bk[n2 - m], xn2);
    tb[m] = v;
  }
  __syncthreads();
  pf::cfftp<true>(B.plan, pool, tb, ch, 1., fuse ? lds : nullptr);
  pf::Cx* bkf = reinterpret_cast<pf::Cx*>(pool + B.bkf);
  for (int64_t i = threadIdx.x; i < n2 / 2 + 1; i += blockDim.x) bkf[i] = tb[i];
}

hipError_t pf_finish(const PfLen& L, const PfLen* dL, double* dpool, double* tmp, hipStream_t st) {
  if (!L.rblue && !L.cblue) return hipSuccess;
  hipLaunchKernelGGL(k_pf_bkf, dim3(1), dim3(kPfThreads), 0, st, dL, dpool, tmp, (int)pf_fuse_on());
  hipError_t e = hipGetLastError();
  if (e == hipSuccess) e = hipStreamSynchronize(st);
  return e;
}

// scipy.signal.resample(x, num), real rows, no window (decoder.py:385-387):
//   X = rfft(x); Y[:N//2+1] = X[:N//2+1] (N = min(num, nx)); an even N's
//   Nyquist bin doubled (num < nx) or halved (num > nx) by numpy's complex
//   multiply with (s + 0j); y = irfft(Y, num) * (num / nx)
// One workgroup per row (rows b = blockIdx.x, + gridDim.x ...); slot: the
// row buffer c (max(nx, num)) then the transforms' scratch.
__global__ __launch_bounds__(kPfThreads) void k_pf_resample(const PfLen* __restrict__ Lx, const double* poolx,
                                                            const PfLen* __restrict__ Ly, const double* pooly,
                                                            const double* __restrict__ x, int64_t nx,
                                                            double* __restrict__ y, int64_t num, int64_t batch,
                                                            double* slots, int64_t slot_doubles, double fct,
                                                            double scale, int fuse) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  pf::Cx* tl = fuse ? lds : nullptr;
  double* c = slots + (size_t)blockIdx.x * slot_doubles;
  double* scr = c + pf_even(std::max(nx, num));
  const int64_t N = std::min(num, nx), nyq = N / 2 + 1;
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    const double* xr = x + (size_t)b * nx;
    for (int64_t i = threadIdx.x; i < nx; i += blockDim.x) c[i] = xr[i];
    __syncthreads();
    pf::pf_r2hc(*Lx, poolx, c, pf::pf_scratch(*Lx, scr, tl), 1.0);
    // halfcomplex of x (c) -> halfcomplex of Y (into the scratch, then back to c)
    double* yh = scr;
    for (int64_t i = threadIdx.x; i < num; i += blockDim.x) {
      // position i of irfft's input: bin k, real (odd i or 0) / imaginary part
      const int64_t k = (i + 1) / 2;
      const bool im = i > 0 && (i & 1) == 0;
      double v = 0.0;
      if (k < nyq) {
        // bin k of X = rfft(x): (c[2k-1], c[2k]); bin 0 and an even nx's nx/2: (c, +0)
        double xr2, xi2;
        if (k == 0) { xr2 = c[0]; xi2 = 0.0; }
        else if (2 * k == nx) { xr2 = c[nx - 1]; xi2 = 0.0; }
        else { xr2 = c[2 * k - 1]; xi2 = c[2 * k]; }
        if (N % 2 == 0 && 2 * k == N && num != nx) {
          const double s = num < nx ? 2.0 : 0.5;
          const double r = xr2, q = xi2;
          xr2 = __builtin_fma(r, s, -(q * 0.0));
          xi2 = __builtin_fma(r, 0.0, q * s);
        }
        v = im ? xi2 : xr2;
      }
      yh[i] = v;
    }
    __syncthreads();
    for (int64_t i = threadIdx.x; i < num; i += blockDim.x) c[i] = yh[i];
    __syncthreads();
    pf::pf_hc2r(*Ly, pooly, c, pf::pf_scratch(*Ly, scr, tl), fct);
    double* yr = y + (size_t)b * num;
    for (int64_t i = threadIdx.x; i < num; i += blockDim.x) yr[i] = c[i] * scale;
    __syncthreads();
  }
}

hipError_t launch_pf_resample(const PfLen* dLx, const double* poolx, const PfLen* dLy, const double* pooly,
                              const double* x, int64_t nx, double* y, int64_t num, int64_t batch, double* slots,
                              int64_t slot_doubles, int n_slots, double fct, double scale, hipStream_t st) {
  if (batch < 1) return hipSuccess;
  const unsigned g = (unsigned)std::min<int64_t>(batch, n_slots);
  hipLaunchKernelGGL(k_pf_resample, dim3(g), dim3(kPfThreads), 0, st, dLx, poolx, dLy, pooly, x, nx, y, num, batch,
                     slots, slot_doubles, fct, scale, (int)pf_fuse_on());
  return hipGetLastError();
}

__global__ __launch_bounds__(kPfThreads) void k_pf_hilbert_env(const PfLen* __restrict__ L, const double* pool,
                                                               double* x, int64_t n, int64_t batch, double* slots,
                                                               int64_t slot_doubles, double fct, int stage,
                                                               int fuse) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  pf::Cx* tl = fuse ? lds : nullptr;
  double* slot = slots + (size_t)blockIdx.x * slot_doubles;
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    double* f = x + (size_t)b * n;
    if (stage == 1) {   // diagnostic: the forward real transform alone (halfcomplex)
      pf::pf_r2hc(*L, pool, f, pf::pf_scratch(*L, slot, tl), 1.0);
    } else if (stage == 2) {   // diagnostic: the backward real transform alone
      pf::pf_hc2r(*L, pool, f, pf::pf_scratch(*L, slot, tl), 1.0);
    } else if (tl && pf_hilbert_fusable(*L)) {
      pf::pf_hilbert_env_x(
          *L, pool, [=](int64_t i) { return f[i]; }, [=](int64_t i, double e) { f[i] = e; }, slot, fct, tl);
    } else {
      pf::pf_hilbert_env(*L, pool, f, f, slot, fct, tl);
    }
  }
}

// lean plans (pf_hilbert_lean): the envelope as two kernels, the real
// transform's halfcomplex output parked in the row itself (the FSK exact
// path's E2a / E2b run the same bodies, fsk_exact_kernels.hip)
__global__ __launch_bounds__(kPfThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_pf_rfft_lean(
    const PfLen* __restrict__ L, const double* pool, double* x, int64_t n, int64_t batch, double* slots,
    int64_t slot_doubles) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  double* slot = slots + (size_t)blockIdx.x * slot_doubles;
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    double* f = x + (size_t)b * n;
    pf::pf_rfft_row(*L, pool, pf::RdD{f}, pf::WrD{f}, slot, lds);
  }
}
__global__ __launch_bounds__(kPfThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_pf_env_lean(
    const PfLen* __restrict__ L, const double* pool, double* x, int64_t n, int64_t batch, double* slots,
    int64_t slot_doubles, double fct) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  double* slot = slots + (size_t)blockIdx.x * slot_doubles;
  for (int64_t b = blockIdx.x; b < batch; b += gridDim.x) {
    double* f = x + (size_t)b * n;
    pf::pf_env_row(*L, pool, pf::RdD{f}, pf::WrD{f}, slot, fct, lds);
  }
}

hipError_t launch_pf_hilbert_env(const PfLen* dL, const double* pool, double* x, int64_t n, int64_t batch,
                                 double* slots, int64_t slot_doubles, int n_slots, double fct, bool lean,
                                 hipStream_t st) {
  if (batch < 1) return hipSuccess;
  const unsigned g = (unsigned)std::min<int64_t>(batch, n_slots);
  // AMR_PF_THREADS (diagnostic): a smaller workgroup (the routines take any size)
  static const unsigned nt = [] {
    const char* e = getenv("AMR_PF_THREADS");
    const int v = e ? atoi(e) : 0;
    return (unsigned)(v >= 64 && v <= kPfThreads ? v : kPfThreads);
  }();
  static const int stage = [] { const char* e = getenv("AMR_PF_STAGE"); return e ? atoi(e) : 0; }();
  if (lean && nt == kPfThreads && pf_fuse_on()) {   // (stage 1 / 2: one half alone, for timing)
    if (stage != 2)
      hipLaunchKernelGGL(k_pf_rfft_lean, dim3(g), dim3(kPfThreads), 0, st, dL, pool, x, n, batch, slots, slot_doubles);
    if (stage != 1)
      hipLaunchKernelGGL(k_pf_env_lean, dim3(g), dim3(kPfThreads), 0, st, dL, pool, x, n, batch, slots, slot_doubles,
                         fct);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_pf_hilbert_env, dim3(g), dim3(nt), 0, st, dL, pool, x, n, batch, slots, slot_doubles, fct,
                     stage, (int)pf_fuse_on());
  return hipGetLastError();
}

}  // namespace amr
