// fsk_exact_kernels.hip -- the FSK path's exact recomputation (DESIGN.md §2
// item 6, §3b).
//
// The fast path's envelopes come from FFTs whose rounding is not pocketfft's,
// so a compare bit env_mark > env_space of fsk_demodulate (modem.py:307-315)
// is certain only where the two envelopes differ by more than both FFTs'
// rounding.  F2's last pass flags every stream with a compare inside that
// margin (fft_kernels.hip env_ambiguous: exact digital silence next to
// signal, a DC or near-silent stretch, a genuine near-tie); this file
// recomputes the flagged streams' compare bits the reference's own way, bit
// for bit, at any length:
//   E0 k_exact_list      flag words -> list of flagged streams (ordinals)
//   E1 F1 in list mode   only on plans without keep_z (the natural layout, or
//                        AMR_FSK_KEEPZ=0): the flagged streams' band-pass
//                        filtfilt again (fsk_kernels.hip k_fsk_bandpass2,
//                        scipy's order), z row q = ordinal q's f_mark + i
//                        f_space, because F2 transformed z's dead tiles in
//                        place.  With keep_z (the default on live-layout
//                        plans) F2 left z -- F1's output, already scipy's
//                        filtfilt bit for bit -- whole, and E2 reads it there.
//   E2 k_exact_rfft +    workgroup = row (stream, tone): |scipy.signal.hilbert(f)|
//      k_exact_cenv      as pocketfft + numpy evaluate it (pocketfft_dev.h,
//      (k_exact_env)     every radix and Bluestein), back into z
//   E3 k_exact_bits      bit = env_mark > env_space in the final pass's byte
//                        layout -> xbits, which F3 (k_fsk_decide) reads for a
//                        flagged stream instead of the fast path's bytes
// With nothing flagged (every noisy capture) each kernel reads the count and
// exits.
#include <algorithm>

#include "amr_internal.h"
#include "fsk_exact.h"
#include "pocketfft_dev.h"

namespace amr {

constexpr int kListThreads = 1024;

// E0: the flagged streams in stream order (ordinal q -> stream), and their count
__global__ __launch_bounds__(kListThreads) void k_exact_list(const uint32_t* __restrict__ flags, int64_t nw,
                                                             int32_t* __restrict__ list, int32_t* __restrict__ count) {
  __shared__ int32_t part[kListThreads];
  const int64_t per = (nw + kListThreads - 1) / kListThreads;
  const int64_t w0 = (int64_t)threadIdx.x * per, w1 = min(nw, w0 + per);
  int32_t c = 0;
  for (int64_t w = w0; w < w1; ++w) c += __popc(flags[w]);
  part[threadIdx.x] = c;
  __syncthreads();
  for (int off = 1; off < kListThreads; off <<= 1) {   // inclusive scan
    const int32_t v = (int)threadIdx.x >= off ? part[threadIdx.x - off] : 0;
    __syncthreads();
    part[threadIdx.x] += v;
    __syncthreads();
  }
  int32_t o = part[threadIdx.x] - c;
  for (int64_t w = w0; w < w1; ++w) {
    uint32_t mm = flags[w];
    while (mm) {
      const int bit = __builtin_ctz(mm);
      mm &= mm - 1;
      list[o++] = (int32_t)(w * 32 + bit);
    }
  }
  if (threadIdx.x == kListThreads - 1) *count = part[threadIdx.x];
}

// the first row of workgroup b: with a grid of whole XCD rounds (workgroup b
// on XCD b % 8), rows 2q and 2q + 1 -- the two tones of one stream, each 8
// bytes of every 16-byte z element -- go to workgroups b and b + 8 of the
// same XCD, so both halves of z's lines meet in one L2
__device__ inline int64_t exact_row0(const FskExact& X) {
  const int G = gridDim.x, b = blockIdx.x;
  if (!X.xcd_pair || G % 16 != 0) return b;
  return (int64_t)(b % 8) * (G / 8) + b / 8;
}

// E2: workgroup = row r = 2q + tone: the tone's band-pass output (F1 in list
// mode left ordinal q's z row = f_mark + i f_space) -> the slot, |hilbert| of
// it, back into the same interleaved positions of z
constexpr int kEnvThreads = 512;
__global__ __launch_bounds__(kEnvThreads) void k_exact_env(FskParams p, FskExact X) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  const int64_t cnt = *X.count;
  const int64_t n = p.n;
  double* c = X.slots + (size_t)blockIdx.x * X.slot_doubles;
  if (X.fuse && pf_hilbert_fusable(*X.L)) {   // straight from z and back, every transform in LDS tiles
    for (int64_t r = exact_row0(X); r < 2 * cnt; r += gridDim.x) {
      double* zr = X.rows + (size_t)(r >> 1) * 2 * n + (r & 1);
      pf::pf_hilbert_env_x(
          *X.L, X.pool, [=](int64_t i) { return zr[2 * i]; }, [=](int64_t i, double e) { zr[2 * i] = e; }, c, X.fct,
          lds);
    }
    return;
  }
  for (int64_t r = exact_row0(X); r < 2 * cnt; r += gridDim.x) {
    double* zr = X.rows + (size_t)(r >> 1) * 2 * n + (r & 1);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) c[i] = zr[2 * i];
    __syncthreads();
    pf::pf_hilbert_env(*X.L, X.pool, c, c, c + pf_even(n), X.fct, X.fuse ? lds : nullptr);
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) zr[2 * i] = c[i];
    __syncthreads();
  }
}

// E2, lean plans (pf_hilbert_lean), as two kernels (one holding both halves
// spills registers): E2a the real transform of row r = tone r & 1 of stream
// s into its halfcomplex spectrum, parked in the row's own z elements in
// natural order (element j at 2 j); E2b the spectrum times h, the inverse
// transform and the envelope, back into z in natural order.  LIVE: s =
// list[r >> 1], f read from z's [L | D] layout (sample i at lc_zoff(i)), only
// live samples' envelopes written (E3 reads no others); otherwise s = r >> 1,
// the F1 re-run's natural rows.  Two workgroups per CU (4 waves per SIMD:
// <= 128 VGPRs).
template <bool LIVE>
struct ZRow {
  double* zr;
  LiveCols lc;
  __device__ int64_t at(int i) const { return LIVE ? 2 * lc_zoff(lc, i) : 2 * (int64_t)i; }
};
template <bool LIVE>
__device__ inline ZRow<LIVE> zrow(const FskParams& p, const FskExact& X, int64_t r) {
  const int64_t s = LIVE ? (int64_t)X.list[r >> 1] : (r >> 1);
  return ZRow<LIVE>{X.rows + (size_t)s * 2 * p.n + (r & 1), X.lc};
}

template <bool LIVE>
__global__ __launch_bounds__(kEnvThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_exact_rfft(FskParams p,
                                                                                                     FskExact X) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  const int64_t cnt = *X.count;
  double* slot = X.slots + (size_t)blockIdx.x * X.slot_doubles;
  for (int64_t r = exact_row0(X); r < 2 * cnt; r += gridDim.x) {
    const ZRow<LIVE> z = zrow<LIVE>(p, X, r);
    // the halfcomplex spectrum parked in natural order (the row's z elements
    // are free once the first group has read them)
    pf::pf_rfft_row(
        *X.L, X.pool, [=](int i) { return z.zr[z.at(i)]; }, [=](int i, double v) { z.zr[2 * (int64_t)i] = v; }, slot,
        lds);
  }
}

template <bool LIVE>
__global__ __launch_bounds__(kEnvThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_exact_cenv(FskParams p,
                                                                                                     FskExact X) {
  __shared__ pf::Cx lds[2 * kPfTileElems];
  const int64_t cnt = *X.count;
  double* slot = X.slots + (size_t)blockIdx.x * X.slot_doubles;
  for (int64_t r = exact_row0(X); r < 2 * cnt; r += gridDim.x) {
    const ZRow<LIVE> z = zrow<LIVE>(p, X, r);
    auto fget = [=](int j) { return z.zr[2 * (int64_t)j]; };
    if (LIVE && X.live_only) {   // envelopes in natural order too, the live samples only (E3 reads no others)
      const LiveCols lc = z.lc;
      pf::pf_env_row(
          *X.L, X.pool, fget,
          [=](int i, double e) {
            const int j2 = lc_div(i, lc.inv_n1);
            bool live;
            (void)lc_col_pos(lc, i - j2 * lc.n1, live);
            if (live) z.zr[2 * (int64_t)i] = e;
          },
          slot, X.fct, lds);
    } else {
      pf::pf_env_row(*X.L, X.pool, fget, [=](int i, double e) { z.zr[2 * (int64_t)i] = e; }, slot, X.fct, lds);
    }
  }
}

// E3: the compare bits of flagged stream s in the final pass's byte layout:
// byte (c0 / 8) * n2 + kk holds columns c0 .. c0 + 7 of row kk (column c ->
// sample col(c) + n1 * kk; col = the live columns or all)
constexpr int kBitsThreads = 256;
__global__ __launch_bounds__(kBitsThreads) void k_exact_bits(FskParams p, FskExact X) {
  const int64_t cnt = *X.count;
  const int64_t n = p.n;
  const int ncol = p.lc.on ? p.lc.nl : (int)p.rn1;
  const int64_t n2 = p.rn2, n1 = p.lc.on ? p.lc.n1 : p.rn1;
  const int64_t nbytes = (int64_t)((ncol + 7) >> 3) * n2;
  if (X.count_host && blockIdx.x == 0 && threadIdx.x == 0) *X.count_host = (int32_t)cnt;
  for (int64_t q = blockIdx.x; q < cnt; q += gridDim.x) {
    const int64_t st = X.list[q];
    // (env_mark, env_space) in natural sample order: z of stream st (live
    // layout, E2 parked them so), or the ordinal row q (natural layout)
    const double2* e = reinterpret_cast<const double2*>(X.rows) + (size_t)(X.live ? st : q) * n;
    uint8_t* ob = X.xbits + (size_t)st * p.bits_stride;
    for (int64_t qb = threadIdx.x; qb < nbytes; qb += blockDim.x) {
      const int64_t cb = qb / n2, kk = qb - cb * n2;
      unsigned byte = 0;
      for (int t = 0; t < 8; ++t) {
        const int c = (int)cb * 8 + t;
        if (c >= ncol) break;
        const int64_t col = p.lc.on ? lc_live_col(p.lc, c) : c;
        const int64_t i = col + n1 * kk;
        if (i < n && e[i].x > e[i].y) byte |= 1u << t;
      }
      ob[qb] = (uint8_t)byte;
    }
  }
}

hipError_t launch_fsk_exact_list(int64_t B, const FskExact& X, hipStream_t st) {
  if (B < 1) return hipSuccess;
  hipLaunchKernelGGL(k_exact_list, dim3(1), dim3(kListThreads), 0, st, X.flags, (B + 31) / 32, X.list, X.count);
  return hipGetLastError();
}

hipError_t launch_fsk_exact_env(int64_t B, const FskParams& p, const FskExact& X, hipStream_t st, bool env) {
  if (B < 1) return hipSuccess;
  // a persistent grid no larger than what is resident at once: a workgroup
  // beyond that would start its rows only after a resident one finished all of
  // its own
  auto resident = [](const void* k) {
    int dev = 0, per_cu = 0, cus = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 256;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k, kEnvThreads, 0) != hipSuccess ||
        hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 256;
    return std::max(1, per_cu * cus);
  };
  static const int res_full = resident((const void*)k_exact_env),
                   res_lean = std::min(resident((const void*)k_exact_rfft<true>), resident((const void*)k_exact_cenv<true>));
  // (FskExact count_hint) two rows per stream, whole XCD rounds of 16, at
  // least kIdleGrid; AMR_FSK_E2_GRID=G (A/B): at most G workgroups
  static const int e2_grid = [] { const char* e = std::getenv("AMR_FSK_E2_GRID"); return e ? std::max(1, atoi(e)) : 1 << 30; }();
  constexpr int64_t kIdleGrid = 16;
  const int64_t want = std::max(kIdleGrid, (2 * std::max<int64_t>(X.count_hint, 0) + 15) / 16 * 16);
  const dim3 gl((unsigned)std::min<int64_t>({X.n_slots, res_lean, e2_grid, want}));
  if (!env) {
    // (diagnostic: the envelope kernels skipped)
  } else if (X.live) {   // the plan guarantees a lean plan (fsk_api.cpp keep_z)
    hipLaunchKernelGGL(k_exact_rfft<true>, gl, dim3(kEnvThreads), 0, st, p, X);
    hipLaunchKernelGGL(k_exact_cenv<true>, gl, dim3(kEnvThreads), 0, st, p, X);
  } else if (X.lean) {
    hipLaunchKernelGGL(k_exact_rfft<false>, gl, dim3(kEnvThreads), 0, st, p, X);
    hipLaunchKernelGGL(k_exact_cenv<false>, gl, dim3(kEnvThreads), 0, st, p, X);
  } else
    hipLaunchKernelGGL(k_exact_env, dim3((unsigned)std::min(X.n_slots, res_full)), dim3(kEnvThreads), 0, st, p, X);
  hipLaunchKernelGGL(k_exact_bits, dim3((unsigned)std::min<int64_t>(B, 256)), dim3(kBitsThreads), 0, st, p, X);
  return hipGetLastError();
}

}  // namespace amr
