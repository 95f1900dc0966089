// pocketfft.h -- plans of the device restatement of pocketfft, the FFT library
// scipy.fft runs (scipy 1.15.3's bundled pocketfft C++ header), for the two
// reference steps whose results depend on its exact rounding:
//   |scipy.signal.hilbert(f)|      modem.fsk_demodulate (modem.py:309, 315):
//                                  the FSK exact path (fsk_exact_kernels.hip)
//   scipy.signal.resample(x, num)  decoder.decode_wav_file (decoder.py:385-387)
// The algorithm is the one oracle/amr_pocketfft.c restates and pins bit for bit
// against scipy on every length 1..2000 (tests/test_oracle_golden.py); the
// plans here are built on the host by the same rules (pocketfft_plan.cpp) and
// executed by pocketfft_dev.h, one workgroup per transform, consecutive passes
// fused through LDS tiles where the plan's groups allow.
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
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <vector>

namespace amr {

constexpr int kPfMaxF = 32;   // factors of one plan (a length < 2^31 has at most 30)
constexpr int64_t kPfMaxLen = (int64_t)1 << 27;   // longest row the device transforms take
// a real row's doubles rounded up to even: complex scratch placed after a row
// stays 16-byte aligned (pocketfft_dev.h Cx is loaded and stored as one b128)
__host__ __device__ inline int64_t pf_even(int64_t n) { return (n + 1) & ~(int64_t)1; }

// x / d for 0 <= x < 2^31 by multiply-high (pocketfft_dev.h FDiv): m =
// floor(2^32 (2^l - d) / d) + 1, l = ceil(log2 d); built on the host for every
// divisor the fused tile loops use, so no division is emulated on the device
struct PfDiv {
  uint32_t m;
  int32_t l, d;
};
inline PfDiv pf_div(int64_t d) {
  PfDiv r{};
  r.d = (int32_t)(d < 1 ? 1 : d);
  r.l = 0;
  while (((int64_t)1 << r.l) < r.d) ++r.l;
  r.m = (uint32_t)(((((uint64_t)1 << 32) * (((uint64_t)1 << r.l) - (uint64_t)r.d)) / (uint64_t)r.d) + 1);
  return r;
}

// one factor of a plan: radix ip, l1 = product of the factors before it,
// ido = len / (l1 * ip); tw / tws: offsets (in doubles) of its twiddles and of
// the generic passes' extra table in the plan's pool, -1 when absent.
// dv: the pass's divisors inside its fused group -- complex: [0] ido / D;
// real blocks: [0] l1 / L, [1] (ido - 1) / 2, [2] their product; real pair
// tiles: [0] B = ido / D, [1] B + 1
struct PfFact {
  int64_t ip, l1, ido, tw, tws;
  PfDiv dv[3];
  int32_t l1l;   // l1 / L inside its fused group (complex, real blocks)
};

// LDS-fused execution of consecutive complex passes (pocketfft_dev.h
// cgroup): passes f0 .. f0 + nf - 1 with radix product P, the last one's ido
// D and the first one's l1 L (len = L * P * D).  A tile is Qi consecutive
// residues i (mod D) times Qk consecutive blocks k: its Q = Qi * Qk columns
// of P elements (i + D (j + P k), j < P) go through every pass of the group
// in LDS and come out at i + D (k + L j) -- the same butterflies, in the same
// order, as the passes run one by one over the whole array.
constexpr int kPfTileElems = 2048;   // complex elements per LDS buffer (32 KiB; two buffers)
constexpr int kPfMaxGroupP = 512;    // radix product of a group (>= 4 columns per tile)
// a two-group complex plan's hand-off rows (D >= kPfPadMinD complex) padded to
// whole kPfPadC-complex (128-byte) lines where the caller has the room
constexpr int kPfPadC = 8, kPfPadMinD = 64;
// rfftp forward (r2hc) groups, in executed order (ido growing): passes
// f0, f0 - 1, ..., f0 - nf + 1; D = the first one's ido, L = the last one's l1;
// a multi-pass group couples every residue mod D, so a tile is Qk whole
// blocks k of D * P reals (read at a + D (k + L w), written to k D P + ...).
// Q = 0 marks a pass run unfused over the whole array (too large a block, or
// a generic radix).  Q = 2: a "pair" group -- the trailing passes from an
// even ido D on (radf4 / radf2 only), L = 1, P = len / D; a tile is Qk pair
// classes {p, D/2 - p} (residues 2p - 1, 2p and their mirrors) or the class
// {0, D - 1}, times all P blocks: reads and writes a + D w.
constexpr int kPfTileDoubles = 2 * kPfTileElems;
constexpr int kPfMinRun = 16;        // doubles a tile reads contiguously, at least
// dv (host-built divisors of the group's tile loops) -- complex: P, Q, Qi,
// the last i-tile's qi, Qk, the last k-tile's qk; real blocks: D, Qk, the
// last tile's qk; pair tiles: R and R / 2 of the special tile, a full tile
// and the last tile
struct PfGroup {
  int f0, nf;
  int64_t P, D, L;
  int Q, Qi, Qk;
  PfDiv dv[8];   // (complex: [6] the i-tile count, for the tile index split; [7] D)
};

// an FFTPACK-style plan (pocketfft's cfftp or rfftp); fused: the passes are
// grouped (g[0..ng)): cfftp when every radix is hard-coded, rfftp (forward)
// always
struct PfPasses {
  int64_t len;
  int nf;
  PfFact f[kPfMaxF];
  int fused, ng;
  PfGroup g[kPfMaxF];
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

// the shape of pocketfft's transforms for scipy.signal.hilbert at length n
// (its real forward and complex inverse FFT): whether either runs Bluestein,
// the length it then transforms (n otherwise) and that length's largest
// prime factor (the widest radix pass) -- for F2's FFT rounding bound
void pf_hilbert_shape(int64_t n, bool* blue, int64_t* n2, int64_t* maxp);

// AMR_PF_FUSE=0 (A/B switch): run the complex transforms pass by pass
// instead of through the LDS-fused groups; default on
bool pf_fuse_on();

// whether |hilbert| of a length-L.n row runs every transform LDS-fused
// (pf_hilbert_env_x), and whether with hard-coded radices only (the lean
// kernels, no generic or unfused fallback code)
__host__ __device__ inline bool pf_hilbert_fusable(const PfLen& L) {
  return !L.rblue && !L.cblue && L.r.fused && L.c.fused && L.r.nf > 0;
}
__host__ __device__ inline bool pf_hilbert_lean(const PfLen& L) {
  if (!pf_hilbert_fusable(L)) return false;
  for (int k = 0; k < L.r.nf; ++k)
    if (L.r.f[k].ip > 5) return false;
  return true;
}

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
                                 double* slots, int64_t slot_doubles, int n_slots, double fct, bool lean,
                                 hipStream_t st);

}  // namespace amr
