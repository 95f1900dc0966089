// fsk_api.cpp -- C ABI of the FSK demodulator and the FFT/Hilbert entry
// points (include/amr.h).  Host code; compiled by hipcc.
//
// Pipeline per call (all on the plan's stream):
//   F1  k_fsk_bandpass          x -> z = f_mark + i f_space           [B][n] c128
//   F2  H[z] = IFFT_n(-i sgn(k) FFT_n(z)) in three passes z -> u -> v -> cmp,
//       the last forming both envelopes: bit = |a_mark| > |a_space|   [B][n/8] u8
//   F3  k_fsk_decide + k_sync_pack  cmp bits -> words -> bytes
// A length that is not 5-smooth runs each FFT_n as a Bluestein convolution of
// length M (u, v then hold M-long rows).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "amr_internal.h"
#include "api_common.h"
#include "fsk_exact.h"
#include "fft.h"
#include "iir_design.h"
#include "split_strict.h"

namespace amr {
hipError_t launch_fsk_bandpass(int, const void*, int64_t, int64_t, double*, double2*, const FskParams&,
                               const FskIir&, hipStream_t);
hipError_t launch_fsk_decide(const uint8_t*, uint32_t*, int64_t, const FskParams&, hipStream_t);
hipError_t launch_fsk_split(int, const void*, int64_t, int64_t, double2*, const FskParams&, const FskIir&,
                            const FskSplit&, hipStream_t);
int64_t fsk_bandpass_scratch_bytes(int64_t n_streams, int64_t n, int pad);
hipError_t launch_sync_pack(const uint32_t*, int64_t, int64_t, int64_t, uint8_t*, int64_t, int64_t*, int64_t*,
                            hipStream_t);
}  // namespace amr

using namespace amr;

namespace {

// Device FFT of one logical length n, run as one of
//   two-pass   M = n = n1 * n2 (launch_fft / launch_fft_filter: the fused paths)
//   six-step   M = n = L1 * L2 past the two-pass limit: transpose, L2-point
//              row FFTs, twiddle-transpose, L1-point row FFTs, transpose
//   Bluestein  n not plannable: a length-M circular convolution, M >= 2n-1,
//              itself two-pass or six-step
// Plain-order epilogues after a six-step / Bluestein transform go through the
// Bluestein post kernel with a unit chirp.
struct FftPlan {
  int64_t n = 0;
  int64_t M = 0;                 // transform length run: n, or the Bluestein length
  bool bluestein = false;
  bool six = false;              // M runs six-step
  FftDesc d{};                   // length M (two-pass)
  FftDesc d1{}, d2{};            // lengths L1, L2 (six-step)
  int64_t L1 = 0, L2 = 0;
  const double2* tw6_lo = nullptr;   // W_M^t, t < 256
  const double2* tw6_hi = nullptr;   // W_M^(256 t)
  const double2* chirp = nullptr;    // Bluestein chirp, or all ones (six-step, plain epilogues)
  const double2* bhat = nullptr;     // FFT_M(bw) (two-pass Bluestein filter table)
  const double2* bhat_c = nullptr;   // conj(FFT_M(bw)) (six-step Bluestein: applied by the post kernel)
  double2* s1 = nullptr;             // six-step scratch [max_batch][M] x 2
  double2* s2 = nullptr;
  int64_t max_batch = 0;
  std::vector<void*> allocs;
};

void fft_plan_free(FftPlan& f) {
  for (void* p : f.allocs)
    if (p) (void)hipFree(p);
  f.allocs.clear();
  f.s1 = f.s2 = nullptr;
}

// device copy of interleaved host values
hipError_t upload(FftPlan& f, const std::vector<double>& h, const double2** out) {
  void* p = nullptr;
  hipError_t e = hipMalloc(&p, h.size() * 8 + 16);
  if (e != hipSuccess) return e;
  f.allocs.push_back(p);
  e = hipMemcpy(p, h.data(), h.size() * 8, hipMemcpyHostToDevice);
  *out = static_cast<const double2*>(p);
  return e;
}

// two-pass descriptor of length L (fft_split must succeed)
int desc_init(FftPlan& f, FftDesc& d, int64_t L) {
  int n1 = 0, n2 = 0;
  if (!fft_split(L, n1, n2)) return fail(AMR_E_INVALID, "FFT length " + std::to_string(L) + " does not split");
  const int64_t nhi = (L + 255) / 256;
  std::vector<double> host;
  auto put = [&](const std::vector<double>& w) { host.insert(host.end(), w.begin(), w.end()); };
  put(twiddles(n2, n2));
  put(twiddles(n1, n1));
  put(twiddles(L, 256));
  put(twiddles(L, nhi, 256));
  const double2* t = nullptr;
  HIP_TRY(upload(f, host, &t));
  d.n = L;
  d.n1 = n1;
  d.n2 = n2;
  if (!fill_fft_len(d.a, n2, t) || !fill_fft_len(d.c, n1, t + n2))
    return fail(AMR_E_INVALID, "FFT factor plan failed for n=" + std::to_string(L));
  d.tw_lo = t + n2 + n1;
  d.tw_hi = t + n2 + n1 + 256;
  return AMR_OK;
}

// X = FFT_M(in) (or the true inverse) by six steps; out may alias in; s1, s2 scratch.
hipError_t six_fft(const FftPlan& f, const double2* in, double2* out, int64_t batch, bool inverse, hipStream_t st) {
  if (batch > f.max_batch) return hipErrorInvalidValue;
  const int64_t L1 = f.L1, L2 = f.L2;
  // in[j1 + L1 j2] = [j2][j1] -> s1[j1][j2]
  hipError_t e = launch_transpose(in, f.s1, L2, L1, batch, nullptr, nullptr, false, st);
  // L2-point transforms of every row j1 -> s1[j1][k2]
  if (e == hipSuccess) e = launch_fft(f.s1, f.s2, f.s1, f.d2, batch * L1, inverse, st);
  // times W_M^(j1 k2), -> s2[k2][j1]
  if (e == hipSuccess) e = launch_transpose(f.s1, f.s2, L1, L2, batch, f.tw6_lo, f.tw6_hi, inverse, st);
  // L1-point transforms of every row k2 -> s2[k2][k1]
  if (e == hipSuccess) e = launch_fft(f.s2, f.s1, f.s2, f.d1, batch * L2, inverse, st);
  // X[k2 + L2 k1] = out[k1][k2]
  if (e == hipSuccess) e = launch_transpose(f.s2, out, L2, L1, batch, nullptr, nullptr, false, st);
  return e;
}

// IFFT_M(FFT_M(a) * FFT_M(bw)) in place in a (Bluestein's convolution), six-step
hipError_t six_conv(const FftPlan& f, double2* a, double2* tmp, int64_t batch, hipStream_t st) {
  FftEpi store{};
  store.mode = kStore;
  store.n = f.M;
  hipError_t e = six_fft(f, a, a, batch, false, st);
  if (e == hipSuccess) e = launch_bs_post(a, a, f.bhat_c, f.M, f.M, batch, false, store, st);   // * FFT(bw)
  if (e == hipSuccess) e = six_fft(f, a, tmp, batch, true, st);
  return e;
}

// How FFT_n runs (host only): two-pass (M = n = n1 * n2), six-step (M = n =
// L1 * L2) or Bluestein over a two-pass / six-step M.  False: no plan.
struct FftShape {
  int64_t M = 0;
  bool bluestein = false, six = false;
  int n1 = 0, n2 = 0;            // the two-pass split of M (when !six)
  int64_t L1 = 0, L2 = 0;        // the six-step split of M (when six)
};
bool fft_shape(int64_t n, FftShape& sh) {
  int a = 0, b = 0;
  if (fft_split(n, a, b)) {
    sh.M = n;
  } else if (fft_six_split(n, sh.L1, sh.L2)) {
    sh.M = n;
    sh.six = true;
  } else {
    sh.bluestein = true;
    sh.M = fft_good_size(2 * n - 1);
    if (sh.M < 0) return false;
    if (!fft_split(sh.M, a, b)) {
      if (!fft_six_split(sh.M, sh.L1, sh.L2)) return false;
      sh.six = true;
    }
  }
  if (!sh.six) fft_split(sh.M, sh.n1, sh.n2);
  return true;
}

// Plans FFT_n for up to max_batch rows; needs the stream for the Bluestein kernel FFT.
int fft_plan_init(FftPlan& f, int64_t n, hipStream_t st, int64_t max_batch) {
  static std::once_flag smem_once;
  static hipError_t smem_err = hipSuccess;
  std::call_once(smem_once, [] { smem_err = fft_configure_smem(); });
  HIP_TRY(smem_err);
  f.n = n;
  f.max_batch = max_batch;
  FftShape sh;
  if (!fft_shape(n, sh)) return fail(AMR_E_INVALID, "no FFT plan for length " + std::to_string(n));
  f.M = sh.M;
  f.bluestein = sh.bluestein;
  f.six = sh.six;
  const int64_t L1 = sh.L1, L2 = sh.L2;
  const int64_t M = f.M;
  if (f.six) {
    f.L1 = L1;
    f.L2 = L2;
    if (int rc = desc_init(f, f.d1, L1)) return rc;
    if (int rc = desc_init(f, f.d2, L2)) return rc;
    const int64_t nhi = (M + 255) / 256;
    std::vector<double> host = twiddles(M, 256);
    const std::vector<double> hi = twiddles(M, nhi, 256);
    host.insert(host.end(), hi.begin(), hi.end());
    const double2* t = nullptr;
    HIP_TRY(upload(f, host, &t));
    f.tw6_lo = t;
    f.tw6_hi = t + 256;
    void* p = nullptr;
    HIP_TRY(hipMalloc(&p, (size_t)(max_batch * M * 16)));
    f.allocs.push_back(p);
    f.s1 = static_cast<double2*>(p);
    HIP_TRY(hipMalloc(&p, (size_t)(max_batch * M * 16)));
    f.allocs.push_back(p);
    f.s2 = static_cast<double2*>(p);
  } else {
    if (int rc = desc_init(f, f.d, M)) return rc;
  }
  if (!f.bluestein && !f.six) return AMR_OK;
  std::vector<double> w((size_t)(2 * n));
  if (f.bluestein) {
    // chirp w_j = exp(i pi j^2 / n); j^2 reduced mod 2n keeps the angle exact
    for (int64_t j = 0; j < n; ++j) {
      const int64_t r = (j * j) % (2 * n);
      const double ang = M_PI * (double)r / (double)n;
      w[(size_t)(2 * j)] = std::cos(ang);
      w[(size_t)(2 * j + 1)] = std::sin(ang);
    }
  } else {
    for (int64_t j = 0; j < n; ++j) w[(size_t)(2 * j)] = 1.0;   // unit chirp: plain epilogues
  }
  HIP_TRY(upload(f, w, &f.chirp));
  if (!f.bluestein) return AMR_OK;
  // convolution kernel bw[m] = w_m, bw[M-m] = w_m (0 < m < n), zero elsewhere; bhat = FFT_M(bw)
  std::vector<double> bw((size_t)(2 * M), 0.0);
  for (int64_t m = 0; m < n; ++m) {
    bw[(size_t)(2 * m)] = w[(size_t)(2 * m)];
    bw[(size_t)(2 * m + 1)] = w[(size_t)(2 * m + 1)];
    if (m > 0) {
      bw[(size_t)(2 * (M - m))] = w[(size_t)(2 * m)];
      bw[(size_t)(2 * (M - m) + 1)] = w[(size_t)(2 * m + 1)];
    }
  }
  const double2* bwd = nullptr;
  HIP_TRY(upload(f, bw, &bwd));
  void* p = nullptr;
  HIP_TRY(hipMalloc(&p, (size_t)M * sizeof(double2)));
  f.allocs.push_back(p);
  double2* bh = static_cast<double2*>(p);
  if (!f.six) {
    double2* tmp = nullptr;
    HIP_TRY(hipMalloc(&tmp, (size_t)M * sizeof(double2)));
    hipError_t e = launch_fft(bwd, tmp, bh, f.d, 1, false, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(tmp);
    HIP_TRY(e);
    f.bhat = bh;
  } else {
    // conj(FFT_M(bw)) by six steps (the post kernel multiplies by conj(w))
    hipError_t e = six_fft(f, bwd, bh, 1, false, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    HIP_TRY(e);
    std::vector<double> hb((size_t)(2 * M));
    HIP_TRY(hipMemcpy(hb.data(), bh, (size_t)M * 16, hipMemcpyDeviceToHost));
    for (int64_t m = 0; m < M; ++m) hb[(size_t)(2 * m + 1)] = -hb[(size_t)(2 * m + 1)];
    HIP_TRY(hipMemcpy(bh, hb.data(), (size_t)M * 16, hipMemcpyHostToDevice));
    f.bhat_c = bh;
  }
  return AMR_OK;
}

// out = FFT_n(in) or IFFT_n(in).  u, v: [batch][M] scratch; in != u; out != v.
hipError_t fft_c2c(const FftPlan& f, const double2* in, double2* u, double2* v, double2* out, int64_t batch,
                   bool inverse, hipStream_t st) {
  if (!f.bluestein) {
    if (f.six) return six_fft(f, in, out, batch, inverse, st);
    return launch_fft(in, u, out, f.d, batch, inverse, st);
  }
  FftEpi store{};
  store.mode = kStore;
  store.n = f.n;        // row stride of `out` (launch_fft_filter sets its own)
  hipError_t e = launch_bs_pre(in, u, f.chirp, f.n, f.M, batch, inverse, st);
  if (f.six) {
    if (e == hipSuccess) e = six_conv(f, u, v, batch, st);
  } else {
    if (e == hipSuccess) e = launch_fft_filter(u, v, u, v, f.d, batch, kMulTab, f.bhat, store, st);
  }
  if (e == hipSuccess) e = launch_bs_post(v, out, f.chirp, f.n, f.M, batch, inverse, store, st);
  return e;
}

// epi(IFFT_n(-i*sgn(k) * FFT_n(in))) = epi(H[in]), the Hilbert transform of
// each row (scipy.signal.hilbert(x).imag for real x).  u, v: [batch][M]
// scratch, in != u, v; a kStore / kEnvOut result lands in hilbert_out(f, u, v).
double2* hilbert_out(const FftPlan& f, double2* u, double2* v) { return (f.bluestein || f.six) ? v : u; }

hipError_t fft_hilbert(const FftPlan& f, const double2* in, double2* u, double2* v, int64_t batch, FftEpi epi,
                       hipStream_t st) {
  epi.n = f.n;
  if (!f.bluestein && !f.six) return launch_fft_filter(in, u, v, u, f.d, batch, kHilbert, nullptr, epi, st);
  const int64_t n = f.n, M = f.M;
  FftEpi store{};
  store.mode = kStore;
  FftEpi hil{};
  hil.mode = kHilbert;
  hil.n = n;
  hipError_t e = hipSuccess;
  if (!f.bluestein) {
    // six-step, M = n: W = -i sgn(k) FFT(in) -> v; IFFT via conj: FFT(conj W) -> v, post conj/scale + epi
    e = six_fft(f, in, u, batch, false, st);
    if (e == hipSuccess) e = launch_bs_post(u, v, f.chirp, n, n, batch, false, hil, st);
    if (e == hipSuccess) e = launch_bs_pre(v, u, f.chirp, n, n, batch, true, st);
    if (e == hipSuccess) e = six_fft(f, u, v, batch, false, st);
    if (e == hipSuccess) e = launch_bs_post(v, v, f.chirp, n, n, batch, true, epi, st);
    return e;
  }
  // forward: W = -i sgn(k) FFT_n(in) -> u (n-long rows)
  e = launch_bs_pre(in, u, f.chirp, n, M, batch, false, st);
  if (f.six) {
    if (e == hipSuccess) e = six_conv(f, u, v, batch, st);
  } else {
    if (e == hipSuccess) e = launch_fft_filter(u, v, u, v, f.d, batch, kMulTab, f.bhat, store, st);
  }
  if (e == hipSuccess) e = launch_bs_post(v, u, f.chirp, n, M, batch, false, hil, st);
  // inverse: epi(IFFT_n(W)) -> v / cmp
  if (e == hipSuccess) e = launch_bs_pre(u, v, f.chirp, n, M, batch, true, st);
  if (f.six) {
    if (e == hipSuccess) e = six_conv(f, v, u, batch, st);
  } else {
    if (e == hipSuccess) e = launch_fft_filter(v, u, v, u, f.d, batch, kMulTab, f.bhat, store, st);
  }
  if (e == hipSuccess) e = launch_bs_post(u, v, f.chirp, n, M, batch, true, epi, st);
  return e;
}

}  // namespace

struct amr_fsk_plan {
  std::mutex mu;
  int device = 0;
  hipStream_t stream = nullptr;
  FskParams p{};
  FskIir f{};
  FftPlan fft{};
  int64_t max_streams = 0;
  int64_t out_cap = 0;
  // HBM scratch
  // natural layout (p.lc.on == 0): z [B][n], u / v [B][M] (u also F1's
  // checkpoint scratch).  Live-column layout (p.lc.on, amr_internal.h
  // LiveCols): z = [B][L | D] (n per stream), u = C [B][nl * n2] -- also F1's
  // checkpoint scratch and, on the host entries, the staged input -- and no v.
  double2* z = nullptr;
  double2* u = nullptr;
  double2* v = nullptr;
  // keep_z (live layout with the exact path): the column pass writes the dead
  // tiles' transform to dd [B][nd * n2] instead of over z's dead columns, so
  // all of z (the band-pass output) survives F2 for the exact path; dd also
  // takes the host entries' staged input (>= 8 B per sample: nd >= n1 / 2).
  // dd (9.6 B per sample at FSK9600) is allocated by the first host entry,
  // which needs a staging buffer anyway; until then the device entries run
  // lean -- dead tiles in place, a flagged stream's F1 re-run from the
  // caller's x (E1) -- so a device-entry plan holds z + C only
  // (AMR_FSK_KEEPZ=1: dd at creation, every call keeps z; =0: never)
  double2* dd = nullptr;
  bool keep_z = false;         // the plan can keep z (dd sized); a call does when dd is allocated
  int64_t dd_bytes = 0;
  int64_t staging_bytes = 0;   // d_x of the host entries (0 with keep_z)
  int64_t u_bytes = 0;
  uint8_t* cmp = nullptr;      // [B][bits_stride] packed compare bits (fft.h fft_bits_stride)
  uint32_t* words = nullptr;   // [B][n_words]
  // the exact path for streams with a compare inside F2's margin (fsk_exact_kernels.hip)
  bool exact_on = false;
  uint32_t* xflags = nullptr;  // [B / 32] F2's flags, bit s of word s / 32 (cleared by F1 every batch)
  double* amb = nullptr;       // [B] F1's ambiguity scale per stream
  int32_t* xlist = nullptr;    // [B] flagged ordinal -> stream, then [1] the count
  int32_t* xcount_host = nullptr;   // host-mapped: the count E3 last saw (FskExact count_hint)
  int32_t* xcount_dev = nullptr;    // its device pointer
  // AMR_FSK_XSTREAM=1 (an A/B, off by default): E0-E3 on a stream of their
  // own at the device's highest priority, ordered by events after F2 and
  // before F3, with the full resident grid every batch.  An exact-path
  // workgroup needs 64 KiB of LDS; from a high-priority queue it takes the
  // next CU that frees that much ahead of the launches in flight.  Measured
  // (profiles/r05_fsk_exact_xstream.txt): alone, fsk9600 36.5-36.8 vs
  // 37.1-37.5 ms/step and a burst of 2048 flagged streams after clean batches
  // 21.8 vs 393 ms of exact stage; but in the default bench process (the
  // PSK headline's 21 streams created first) 39.2-39.9 vs 37.3-37.4 ms/step,
  // two interleaved pairs -- so the plan's own stream stays the default, and
  // the synchronous host entry sizes the grid from the batch's own count
  // (count_sync)
  hipStream_t xstream = nullptr;
  hipEvent_t ev_f2 = nullptr, ev_x = nullptr;
  // the synchronous host entry (amr_fsk_demod_host) reads E0's count on the
  // host before the envelope kernels: none flagged -> E1-E3 are not launched
  // at all; else E2's grid is sized from this batch's own count
  bool count_sync = false;
  // the counts E3 reported before the last kHintDepth launches:
  // E2's grid follows their maximum, so one clean batch between flagged ones
  // does not shrink the grid of the next flagged batch to kIdleGrid
  static constexpr int kHintDepth = 8;
  int32_t hint_hist[kHintDepth]{};
  int hint_pos = 0;
  double* xslots = nullptr;    // [n_slots][slot_doubles] envelope scratch
  uint8_t* xbits = nullptr;    // [B][bits_stride] the flagged streams' exact compare bits
  double* xpool = nullptr;     // pocketfft's twiddle / chirp tables of length n
  PfLen* xL = nullptr;         // pocketfft's plans of length n (device copy)
  bool x_lean = false;         // pf_hilbert_lean: E2 runs the lean fused kernel
  int64_t slot_doubles = 0;
  int n_slots = 0;
  bool ran_exact = false;      // the last call ran the exact path (its count is in xlist[max_streams])
  int exact_mode = 1;          // amr_fsk_plan_set_exact_mode: 0 off, 1 F2's flags, 2 every stream
  int64_t scratch_bytes = 0;
  // the time-split F1 (fsk_kernels.hip FS1-FS3): designed
  // with the plan; used for calls of at most kFskSplitMaxStreams streams
  // (amr_fsk_plan_set_layout overrides); its forward outputs and peaks in
  // split_y1 / split_peak, allocated on the first split call (<= 1024 streams)
  bool split_ok = false;
  int64_t split_w = 0;
  double split_kappa = 0.0, split_hl1 = 0.0, split_tau = 0.0;
  int split_mode = AMR_FSK_LAYOUT_AUTO;
  bool split_now = false;      // this call runs the split F1 (z approximate: no keep_z, E1 re-runs F1)
  bool last_split = false;
  int64_t split_L = 0;
  double* split_y1 = nullptr;
  unsigned long long* split_peak = nullptr;
  int64_t split_cap = 0;       // streams split_y1 / split_peak hold
  int64_t split_alloc = 0;     // their bytes (not in scratch_bytes)
  int64_t split_reserved = 0;  // what amr_fsk_plan_bytes_estimate counts for them (<= 1024 streams)
  // FS0's convolution start states: tables [2][w][6] + [2][w + 1][6] (host
  // copy made with the design), on the device with the zs states in split_cz
  std::vector<double> split_tab_host;
  double* split_cz = nullptr;
  int64_t split_cz_bytes = 0;
  // the split F1's STRICT mode (round 6; split_strict.h strict_design_bp per
  // tone, fsk_kernels.hip FS0-FS2 with ST, KF1-KF2, FS3): designed on the
  // first strict call; its tables, per-stream maxima and scratch in
  // strict_tab / strict_bnd / strict_sc (strict_bytes, not in split_alloc)
  int strict_mode = -1;        // amr_fsk_plan_set_split_strict: 1 on, 0 off, -1 the default
  bool strict_designed = false, strict_ok = false, last_strict = false;
  StrictDesign sdes[2];
  double* strict_tab = nullptr;
  unsigned long long* strict_bnd = nullptr;
  double* strict_sc = nullptr;
  int64_t strict_tab_n = 0, strict_bnd_cap = 0, strict_sc_bytes = 0, strict_bytes = 0;
  GatherGate gate;             // an all-gather still reading this plan's outputs
  // staging for the host API
  void* d_x = nullptr;
  uint8_t* d_out = nullptr;
  int64_t* d_len = nullptr;
  int64_t* d_sync = nullptr;
  double* d_edge = nullptr;    // amr_fsk_demod_host_edges' table [max_streams][2 pad] (with d_out)
  // timing
  bool timing = false;
  hipEvent_t ev[AMR_TF_COUNT][2]{};
  bool ev_used[AMR_TF_COUNT]{};
};

namespace {

void fsk_plan_free(amr_fsk_plan* pl) {
  if (!pl) return;
  (void)hipSetDevice(pl->device);
  if (pl->stream) (void)hipStreamSynchronize(pl->stream);
  gate_free(pl->gate);
  if (pl->xcount_host) (void)hipHostFree(pl->xcount_host);
  for (void* p : {(void*)pl->z, (void*)pl->u, (void*)pl->v, (void*)pl->dd, (void*)pl->cmp, (void*)pl->words, pl->d_x,
                  (void*)pl->d_out, (void*)pl->d_len, (void*)pl->d_sync, (void*)pl->xflags, (void*)pl->amb,
                  (void*)pl->xlist, (void*)pl->xslots, (void*)pl->xbits, (void*)pl->xpool, (void*)pl->xL,
                  (void*)pl->split_y1, (void*)pl->split_peak, (void*)pl->split_cz, (void*)pl->d_edge,
                  (void*)pl->strict_tab, (void*)pl->strict_bnd, (void*)pl->strict_sc})
    if (p) (void)hipFree(p);
  fft_plan_free(pl->fft);
  for (auto& e : pl->ev)
    for (auto& h : e)
      if (h) (void)hipEventDestroy(h);
  if (pl->xstream) (void)hipStreamSynchronize(pl->xstream);
  if (pl->ev_f2) (void)hipEventDestroy(pl->ev_f2);
  if (pl->ev_x) (void)hipEventDestroy(pl->ev_x);
  if (pl->xstream) (void)hipStreamDestroy(pl->xstream);
  if (pl->stream) (void)hipStreamDestroy(pl->stream);
  delete pl;
}

// this call keeps z whole through F2 (dd allocated: see amr_fsk_plan::dd;
// a split call's z is not scipy's, so the exact path re-runs F1 instead)
bool keeps_z(const amr_fsk_plan* pl) { return pl->keep_z && pl->dd != nullptr && !pl->split_now; }

hipError_t mark_fsk(amr_fsk_plan* pl, int slot, int which, hipStream_t st = nullptr) {
  if (!pl->timing) return hipSuccess;
  pl->ev_used[slot] = true;
  return hipEventRecord(pl->ev[slot][which], st ? st : pl->stream);
}

// F1 over the B streams of x -> z (and, with the exact path on, each
// stream's ambiguity scale; the flag words cleared).  Caller holds mu.
constexpr int64_t kFskSplitMaxStreams = 1024;   // AUTO: calls of at most this many streams split

// The split F1's launch geometry: L outputs per chunk (at least
// kFskSplitMinL and w / 4, so warm-ups are at most 4x the useful work, and
// long enough to keep a launch within kFskSplitLanes lanes)
constexpr int64_t kFskSplitMinL = 64;
constexpr int64_t kFskSplitLanes = 65536;
// with FS0's convolution start states (AMR_FSK_SPLIT_CONV=0: the warm-ups):
// chunks of kFskSplitConvMinL..MaxL outputs, about kFskSplitConvChunks (chunk,
// tone) waves per call -- the PSK split's rule (api.cpp kSplitConv*)
constexpr int64_t kFskSplitConvMinL = 128;
constexpr int64_t kFskSplitConvMaxL = 1024;
constexpr int64_t kFskSplitConvChunks = 3072;
// the split F1's strict margin by default (AMR_FSK_SPLIT_STRICT=0 / 1 overrides)
constexpr int kFskStrictDefault = 1;
bool fsk_split_conv_on(const amr_fsk_plan* pl) {
  static const bool env = [] { const char* e = std::getenv("AMR_FSK_SPLIT_CONV"); return !(e && e[0] == '0'); }();
  return env && pl->split_ok && !pl->split_tab_host.empty();
}
// STRICT: AMR_FSK_SPLIT_STRICT=0 / 1 sets the default, amr_fsk_plan_set_split_strict
// a plan's; the bound covers the convolution starts only
bool fsk_split_strict_on(const amr_fsk_plan* pl) {
  static const int env = [] {
    const char* e = std::getenv("AMR_FSK_SPLIT_STRICT");
    return e ? (e[0] == '1' ? 1 : 0) : kFskStrictDefault;
  }();
  const bool want = pl->strict_mode >= 0 ? pl->strict_mode == 1 : env == 1;
  return want && fsk_split_conv_on(pl);
}
FskSplit fsk_split_params(amr_fsk_plan* pl, int64_t B, int64_t L) {
  FskSplit sp{};
  const int64_t m1 = pl->p.n + 2 * (int64_t)pl->p.pad;
  sp.conv = fsk_split_conv_on(pl) ? 1 : 0;
  const int64_t lanes = (2 * B * m1 + kFskSplitLanes - 1) / kFskSplitLanes;
  if (L > 0) sp.L = L;
  else if (sp.conv)
    sp.L = std::max(lanes, std::min(kFskSplitConvMaxL, std::max(kFskSplitConvMinL,
                                                                  (2 * B * m1 + kFskSplitConvChunks - 1) /
                                                                      kFskSplitConvChunks)));
  else sp.L = std::max({kFskSplitMinL, pl->split_w / 4, lanes});
  sp.w = pl->split_w;
  if (L <= 0 && sp.conv && fsk_split_strict_on(pl) && pl->strict_ok)   // chunks on block boundaries
    sp.L = (sp.L + kStrictBlk - 1) / kStrictBlk * kStrictBlk;
  sp.c = (m1 + sp.L - 1) / sp.L;
  sp.tau = pl->split_tau;
  sp.y1 = pl->split_y1;
  sp.peak = pl->split_peak;
  pl->split_L = sp.L;
  return sp;
}

// STRICT: the per-tone designs from FS0's tables (host arithmetic, once) and
// their device copy: per tone kabs [w] | z0abs [w + 1] | W | K12 | HS | GS | TZ
int fsk_strict_prepare(amr_fsk_plan* pl) {
  if (pl->strict_designed) return AMR_OK;
  pl->strict_designed = true;
  pl->strict_ok = false;
  if (!pl->split_ok || pl->split_tab_host.empty()) return AMR_OK;
  const int nt = pl->p.nt;
  const int64_t w = pl->split_w;
  bool ok = true;
  for (int t = 0; t < 2 && ok; ++t) {
    Iir fi{};
    fi.nt = nt;
    for (int i = 0; i < nt; ++i) { fi.b[i] = pl->f.b[t][i]; fi.a[i] = pl->f.a[t][i]; }
    for (int i = 0; i < nt - 1; ++i) fi.zi[i] = pl->f.zi[t][i];
    StrictDesign& d = pl->sdes[t];
    ok = strict_design_bp(fi, pl->split_tab_host.data() + (size_t)t * w * 6,
                          pl->split_tab_host.data() + (size_t)(2 * w + t * (w + 1)) * 6, w, d,
                          strict_detail::responses(fi)) &&
         d.g1x * (d.kx + 2.0 * d.ky) < 0.125;
    d.ok = ok;
  }
  if (!ok) return AMR_OK;
  std::vector<double> tab;
  for (int t = 0; t < 2; ++t)
    for (const std::vector<double>* v : {&pl->sdes[t].kabs, &pl->sdes[t].z0abs, &pl->sdes[t].W, &pl->sdes[t].K12,
                                         &pl->sdes[t].HS, &pl->sdes[t].GS, &pl->sdes[t].TZ})
      tab.insert(tab.end(), v->begin(), v->end());
  HIP_TRY(hipMalloc((void**)&pl->strict_tab, tab.size() * 8));
  HIP_TRY(hipMemcpy(pl->strict_tab, tab.data(), tab.size() * 8, hipMemcpyHostToDevice));
  pl->strict_tab_n = (int64_t)tab.size();
  pl->strict_bytes += (int64_t)tab.size() * 8;
  pl->strict_ok = true;
  return AMR_OK;
}
// STRICT: this call's scratch and maxima for B streams, and sp's strict fields
int ensure_fsk_strict(amr_fsk_plan* pl, FskSplit& sp, int64_t B) {
  // (a diagnostic's forced chunk off block boundaries runs without it)
  if (!sp.conv || !fsk_split_strict_on(pl) || !pl->strict_ok || sp.L % kStrictBlk != 0) return AMR_OK;
  const int64_t m1 = pl->p.n + 2 * (int64_t)pl->p.pad;
  sp.nb1 = (m1 + kStrictBlk - 1) / kStrictBlk;
  sp.sstride = 5 * sp.nb1 + 2 * sp.c;
  const int64_t need = B * 2 * sp.sstride * 8;
  if (pl->strict_sc_bytes < need || !pl->strict_sc) {
    HIP_TRY(hipStreamSynchronize(pl->stream));
    if (pl->strict_sc) (void)hipFree(pl->strict_sc);
    pl->strict_bytes -= pl->strict_sc_bytes;
    pl->strict_sc = nullptr;
    pl->strict_sc_bytes = 0;
    HIP_TRY(hipMalloc((void**)&pl->strict_sc, (size_t)need));
    pl->strict_sc_bytes = need;
    pl->strict_bytes += need;
  }
  if (pl->strict_bnd_cap < B || !pl->strict_bnd) {
    HIP_TRY(hipStreamSynchronize(pl->stream));
    if (pl->strict_bnd) (void)hipFree(pl->strict_bnd);
    pl->strict_bytes -= pl->strict_bnd_cap * 2 * 64;
    pl->strict_bnd = nullptr;
    pl->strict_bnd_cap = 0;
    HIP_TRY(hipMalloc((void**)&pl->strict_bnd, (size_t)(B * 2 * 64)));
    pl->strict_bnd_cap = B;
    pl->strict_bytes += B * 2 * 64;
  }
  sp.strict = 1;
  sp.u2 = 2.0 * 0x1p-53 * (1.0 + 0x1p-50);
  sp.hl1 = pl->split_hl1;
  sp.sc = pl->strict_sc;
  sp.bnd = pl->strict_bnd;
  const double* o = pl->strict_tab;
  for (int t = 0; t < 2; ++t) {
    const StrictDesign& d = pl->sdes[t];
    StrictBp& b = sp.sb[t];
    b.kabs = o;
    o += d.kabs.size();
    b.z0abs = o;
    o += d.z0abs.size();
    b.W = o;
    o += d.W.size();
    b.K12 = o;
    o += d.K12.size();
    b.HS = o;
    o += d.HS.size();
    b.GS = o;
    o += d.GS.size();
    b.TZ = o;
    o += d.TZ.size();
    b.nw = (int)d.W.size();
    b.nk = (int)d.K12.size();
    b.nh = (int)d.HS.size();
    b.nz = (int)d.TZ.size();
    b.k12_off = d.k12_off;
    b.w_tail = d.w_tail;
    b.k12_tail = d.k12_tail;
    b.hs_tail = d.hs_tail;
    b.tz_tail = d.tz_tail;
    b.gam = d.gam;
    b.kx = d.kx;
    b.ky = d.ky;
    b.g1x = d.g1x;
    b.gmax = d.gmax;
    b.hz = d.hz;
    b.tk = d.tk;
    b.zi_sum = d.zi_sum;
    b.zb = d.zb;
  }
  return AMR_OK;
}
// the tables and this call's zs in split_cz (grown as needed; counted in
// split_alloc), then sp's pointers into it
int ensure_split_conv(amr_fsk_plan* pl, FskSplit& sp, int64_t B) {
  if (!sp.conv) return AMR_OK;
  const int64_t tab = (int64_t)pl->split_tab_host.size() * 8;
  const int64_t need = tab + B * 2 * sp.c * 6 * 8;
  if (pl->split_cz_bytes < need || !pl->split_cz) {
    HIP_TRY(hipStreamSynchronize(pl->stream));
    if (pl->split_cz) {
      (void)hipFree(pl->split_cz);
      pl->split_alloc -= pl->split_cz_bytes;
    }
    pl->split_cz = nullptr;
    pl->split_cz_bytes = 0;
    HIP_TRY(hipMalloc((void**)&pl->split_cz, (size_t)need));
    HIP_TRY(hipMemcpy(pl->split_cz, pl->split_tab_host.data(), (size_t)tab, hipMemcpyHostToDevice));
    pl->split_cz_bytes = need;
    pl->split_alloc += need;
  }
  sp.ktab = pl->split_cz;
  sp.z0tab = pl->split_cz + 2 * sp.w * 6;
  sp.zs = pl->split_cz + tab / 8;
  return AMR_OK;
}
int ensure_split_buffers(amr_fsk_plan* pl, int64_t B) {
  if (B <= pl->split_cap) return AMR_OK;
  const int64_t m1 = pl->p.n + 2 * (int64_t)pl->p.pad;
  if (pl->split_y1 || pl->split_peak) {
    HIP_TRY(hipStreamSynchronize(pl->stream));
    (void)hipFree(pl->split_y1);
    (void)hipFree(pl->split_peak);
    pl->split_y1 = nullptr;
    pl->split_peak = nullptr;
    pl->split_alloc = pl->split_cz_bytes;
    pl->split_cap = 0;
  }
  HIP_TRY(hipMalloc(&pl->split_y1, (size_t)(B * 2 * m1 * 8)));
  HIP_TRY(hipMalloc(&pl->split_peak, (size_t)(B * 8)));
  pl->split_cap = B;
  pl->split_alloc = B * (2 * m1 * 8 + 8) + pl->split_cz_bytes;
  return AMR_OK;
}
// does this call run the split F1?  Only with the exact path on (it is what
// makes the split's decisions exact)
bool use_split(const amr_fsk_plan* pl, int64_t B) {
  static const bool env_off = [] { const char* e = std::getenv("AMR_FSK_SPLIT"); return e && e[0] == '0'; }();
  if (!pl->split_ok || !pl->exact_on || pl->exact_mode == 0 || pl->p.n_bits == 0 || B < 1 || B > 65535) return false;
  if (pl->split_mode == AMR_FSK_LAYOUT_SPLIT) return true;
  return pl->split_mode == AMR_FSK_LAYOUT_AUTO && !env_off && B <= kFskSplitMaxStreams;
}

int run_fsk_f1(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, bool exact) {
  FskParams p = pl->p;
  if (!(exact && pl->exact_on && pl->exact_mode != 0)) p.amb = nullptr;
  p.force_exact = pl->exact_mode == 2 ? 1 : 0;
  if (pl->split_now) {
    if (int rc = ensure_split_buffers(pl, B)) return rc;
    if (fsk_split_strict_on(pl))
      if (int rc = fsk_strict_prepare(pl)) return rc;
    FskSplit sp = fsk_split_params(pl, B, 0);
    if (int rc = ensure_split_conv(pl, sp, B)) return rc;
    if (int rc = ensure_fsk_strict(pl, sp, B)) return rc;
    pl->last_strict = sp.strict != 0;
    HIP_TRY(launch_fsk_split(dtype, d_x, x_stride, B, pl->z, p, pl->f, sp, pl->stream));
    return AMR_OK;
  }
  HIP_TRY(launch_fsk_bandpass(dtype, d_x, x_stride, B, reinterpret_cast<double*>(pl->u), pl->z, p, pl->f,
                              pl->stream));
  return AMR_OK;
}

// F2 over the B streams of z: the Hilbert filter, whose last pass forms both
// envelopes, packs the compare bits and flags the streams with a compare
// inside the margin (or, env_out on a natural-layout plan, stores the
// envelopes themselves in hilbert_out(u, v)).
int run_fsk_f2(amr_fsk_plan* pl, int64_t B, bool env_out) {
  FftEpi env{};
  env.mode = env_out ? kEnvOut : kEnvelope;
  env.z = pl->z;
  env.bits = pl->cmp;
  env.bits_stride = pl->p.bits_stride;
  if (!env_out && pl->exact_on && pl->exact_mode != 0) {
    env.amb = pl->amb;
    env.xflags = pl->xflags;
  }
  // one timing slot for the whole Hilbert filter (column, middle and final passes)
  HIP_TRY(mark_fsk(pl, AMR_TF_HILBERT, 0));
  if (pl->p.lc.on) {
    if (env_out) return fail(AMR_E_INVALID, "live-column plan: envelopes go through a natural-layout plan");
    // AMR_FSK_SUBBATCH=S (an A/B experiment): the three
    // passes per sub-batch of S streams (a multiple of 32: the flag words),
    // so a sub-batch's intermediates could stay in the Infinity Cache
    static const int64_t sub = [] {
      const char* e = std::getenv("AMR_FSK_SUBBATCH");
      const int64_t v = e ? atoll(e) : 0;
      return v >= 32 ? v / 32 * 32 : 0;
    }();
    const LiveCols& lc = pl->p.lc;
    const int64_t step = sub > 0 ? sub : B;
    for (int64_t b0 = 0; b0 < B; b0 += step) {
      const int64_t nb = std::min(step, B - b0);
      FftEpi e = env;
      e.z = env.z + b0 * pl->p.n;
      e.bits = env.bits + b0 * env.bits_stride;
      if (e.amb) e.amb += b0;
      if (e.xflags) e.xflags += b0 / 32;
      HIP_TRY(launch_fft_hilbert_live(pl->z + b0 * pl->p.n, pl->u + b0 * (int64_t)lc.nl * lc.n2,
                                      keeps_z(pl) ? pl->dd + b0 * (int64_t)lc.nd * lc.n2 : nullptr, pl->fft.d, nb, lc,
                                      e, pl->stream));
    }
  } else {
    HIP_TRY(fft_hilbert(pl->fft, pl->z, pl->u, pl->v, B, env, pl->stream));
  }
  HIP_TRY(mark_fsk(pl, AMR_TF_HILBERT, 1));
  return AMR_OK;
}

// AMR_FSK_EXACT_LAUNCH=0 (diagnostic A/B only, decisions then NOT exact):
// F1 / F2 keep their margin work, the E0-E3 launches are skipped (=2: E0 and
// E3 only, E2 skipped).  Either way F3 then takes every stream's bits from the
// fast path (run_fsk_back), not from an xbits buffer E2 / E3 never filled.
int exact_launch_mode() {
  static const int launch = [] { const char* e = std::getenv("AMR_FSK_EXACT_LAUNCH"); return e ? atoi(e) : 1; }();
  return launch;
}

// The exact path over F2's flagged streams: with keep_z straight from z (F2
// left it whole), otherwise F1 again over their input x (still resident).
int run_fsk_exact(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride) {
  if (!pl->exact_on || pl->exact_mode == 0) return AMR_OK;
  const int launch = exact_launch_mode();
  if (launch == 0) return AMR_OK;
  FskExact X{};
  X.flags = pl->xflags;
  X.list = pl->xlist;
  X.count = pl->xlist + pl->max_streams;
  X.rows = reinterpret_cast<double*>(pl->z);
  X.live = keeps_z(pl) ? 1 : 0;
  X.lc = pl->p.lc;
  X.slots = pl->xslots;
  X.slot_doubles = pl->slot_doubles;
  X.n_slots = pl->n_slots;
  X.L = pl->xL;
  X.pool = pl->xpool;
  X.fct = (double)(1.0L / (long double)pl->p.n);
  X.xbits = pl->xbits;
  X.fuse = (int)pf_fuse_on();
  X.lean = X.fuse && pl->x_lean;
  static const int xcd_pair = [] { const char* e = std::getenv("AMR_FSK_XCDPAIR"); return !(e && e[0] == '0'); }();
  X.xcd_pair = xcd_pair;
  static const int live_only = [] { const char* e = std::getenv("AMR_FSK_LIVEONLY"); return !(e && e[0] == '0'); }();
  X.live_only = live_only;
  X.count_host = pl->xcount_dev;
  if (pl->xstream && !pl->count_sync) {
    X.count_hint = B;                                   // the full resident grid (see xstream)
  } else if (pl->xcount_host) {
    pl->hint_hist[pl->hint_pos] = *reinterpret_cast<volatile int32_t*>(pl->xcount_host);
    pl->hint_pos = (pl->hint_pos + 1) % amr_fsk_plan::kHintDepth;
    X.count_hint = *std::max_element(pl->hint_hist, pl->hint_hist + amr_fsk_plan::kHintDepth);
  } else {
    X.count_hint = B;
  }
  hipStream_t st = pl->stream;
  const bool xs = pl->xstream && !pl->count_sync;
  if (xs) {
    HIP_TRY(hipEventRecord(pl->ev_f2, pl->stream));
    HIP_TRY(hipStreamWaitEvent(pl->xstream, pl->ev_f2, 0));
    st = pl->xstream;
  }
  HIP_TRY(mark_fsk(pl, AMR_TF_EXACT, 0, st));
  pl->ran_exact = true;
  HIP_TRY(launch_fsk_exact_list(B, X, st));
  if (pl->count_sync) {
    int32_t c = 0;
    HIP_TRY(hipMemcpyAsync(&c, X.count, 4, hipMemcpyDeviceToHost, st));
    HIP_TRY(hipStreamSynchronize(st));
    if (c == 0) {                            // nothing flagged: F3 takes every stream's fast-path bits
      pl->ran_exact = false;
      *pl->xcount_host = 0;
      HIP_TRY(mark_fsk(pl, AMR_TF_EXACT, 1, st));
      return AMR_OK;
    }
    X.count_hint = c;
  }
  if (!X.live) {
    // E1: F1 again over the flagged streams only (list mode), natural z layout
    FskParams p1 = pl->p;
    p1.amb = nullptr;
    p1.lc = LiveCols{};
    p1.xlist = X.list;
    p1.xcount = X.count;
    HIP_TRY(launch_fsk_bandpass(dtype, d_x, x_stride, B, reinterpret_cast<double*>(pl->u), pl->z, p1, pl->f, st));
  }
  HIP_TRY(launch_fsk_exact_env(B, pl->p, X, st, launch != 2));
  HIP_TRY(mark_fsk(pl, AMR_TF_EXACT, 1, st));
  if (xs) {
    HIP_TRY(hipEventRecord(pl->ev_x, pl->xstream));
    HIP_TRY(hipStreamWaitEvent(pl->stream, pl->ev_x, 0));
  }
  return AMR_OK;
}

// F1, F2 (and the exact path) on a device-resident batch: x -> cmp (or the envelopes).  Caller holds mu.
int run_fsk_front(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, bool env_out) {
  if (env_out) pl->split_now = false;        // the envelopes themselves: scipy's F1
  HIP_TRY(mark_fsk(pl, AMR_TF_BANDPASS, 0));
  if (int rc = run_fsk_f1(pl, d_x, dtype, B, x_stride, !env_out)) return rc;
  HIP_TRY(mark_fsk(pl, AMR_TF_BANDPASS, 1));
  if (int rc = run_fsk_f2(pl, B, env_out)) return rc;
  if (env_out) return AMR_OK;
  return run_fsk_exact(pl, d_x, dtype, B, x_stride);
}

int check_fsk_args(amr_fsk_plan* pl, int dtype, int64_t B, int64_t x_stride, int64_t out_stride) {
  if (B < 0 || B > pl->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (dtype_size(dtype) == 0) return fail(AMR_E_INVALID, "unknown dtype");
  if (x_stride < pl->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < pl->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  return AMR_OK;
}

// no decision window (sps // 4 == 0): empty bit string -> b''   (modem.py:320-323)
int fsk_empty_outputs(amr_fsk_plan* pl, int64_t B, int64_t* d_len, int64_t* d_sync) {
  HIP_TRY(gate_wait(pl->gate, pl->stream));
  HIP_TRY(hipMemsetAsync(d_len, 0, (size_t)B * 8, pl->stream));
  HIP_TRY(hipMemsetAsync(d_sync, 0xFF, (size_t)B * 8, pl->stream));
  return AMR_OK;
}

// F3: compare bits -> decided words -> sync + pack.  Caller holds mu.
int run_fsk_back(amr_fsk_plan* pl, int64_t B, uint8_t* d_out, int64_t out_stride, int64_t* d_len, int64_t* d_sync) {
  hipStream_t st = pl->stream;
  HIP_TRY(mark_fsk(pl, AMR_TF_DECIDE, 0));
  // a flagged stream's bits come from xbits only when this call's E0-E3 wrote
  // them (exact mode 0 leaves the flag words of an earlier call untouched;
  // the diagnostic launch modes leave xbits unwritten)
  FskParams p = pl->p;
  if (!pl->ran_exact || exact_launch_mode() != 1) p.xflags = nullptr;
  HIP_TRY(launch_fsk_decide(pl->cmp, pl->words, B, p, st));
  HIP_TRY(gate_wait(pl->gate, st));             // the outputs: after any gather still reading them
  HIP_TRY(launch_sync_pack(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync, st));
  HIP_TRY(mark_fsk(pl, AMR_TF_DECIDE, 1));
  return AMR_OK;
}

// the call's odd-extension table (odd_ext.h) in the plan's FskParams for the
// launches of one call (F1, its split form and the exact path's F1 re-run
// copy pl->p); cleared when the call returns.  Caller holds mu.
struct EdgeScope {
  FskParams& p;
  EdgeScope(FskParams& q, const double* e) : p(q) { p.edge = e; }
  ~EdgeScope() { p.edge = nullptr; }
};

// d_edge: [B][2 pad] for a raw-integer capture (include/amr.h
// amr_fsk_demod_host_edges), or null
int run_fsk(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, uint8_t* d_out,
            int64_t out_stride, int64_t* d_len, int64_t* d_sync, const double* d_edge = nullptr) {
  if (int rc = check_fsk_args(pl, dtype, B, x_stride, out_stride)) return rc;
  EdgeScope edge_scope(pl->p, d_edge);
  for (bool& u : pl->ev_used) u = false;
  pl->ran_exact = false;
  pl->split_now = use_split(pl, B);
  pl->last_split = pl->split_now;
  if (B == 0) return AMR_OK;
  if (pl->p.n_bits == 0) return fsk_empty_outputs(pl, B, d_len, d_sync);
  HIP_TRY(mark_fsk(pl, AMR_TF_LAUNCH, 0));
  if (int rc = run_fsk_front(pl, d_x, dtype, B, x_stride, false)) return rc;
  if (int rc = run_fsk_back(pl, B, d_out, out_stride, d_len, d_sync)) return rc;
  HIP_TRY(mark_fsk(pl, AMR_TF_LAUNCH, 1));
  return AMR_OK;
}

// Where the host entries stage the input (max_streams rows of up to 8 B per
// sample): dd with keep_z (the column pass overwrites it after F1 read it),
// else d_x, where it stays for the exact path's F1 re-run after F2.
int staging_buffer(amr_fsk_plan* pl, void** buf) {
  if (pl->keep_z) {
    if (!pl->dd) {
      HIP_TRY(hipMalloc(&pl->dd, (size_t)pl->dd_bytes));
      pl->scratch_bytes += pl->dd_bytes;
    }
    *buf = pl->dd;
    return AMR_OK;
  }
  if (!pl->d_x) HIP_TRY(hipMalloc(&pl->d_x, (size_t)(pl->max_streams * pl->p.n * 8)));
  *buf = pl->d_x;
  return AMR_OK;
}
int stage_input(amr_fsk_plan* pl, const void* x, int dtype, int64_t B, int64_t x_stride, void** staged) {
  const int64_t es = dtype_size(dtype);
  const int64_t n = pl->p.n;
  if (int rc = staging_buffer(pl, staged)) return rc;
  return copy_batch_h2d(*staged, x, n * es, x_stride * es, B, pl->stream);
}

// the host entries' output staging and the edge table (amr_fsk_demod_host_edges)
int ensure_out_staging(amr_fsk_plan* pl) {
  if (pl->d_out) return AMR_OK;
  HIP_TRY(hipMalloc(&pl->d_out, (size_t)(pl->max_streams * pl->out_cap)));
  HIP_TRY(hipMalloc(&pl->d_len, (size_t)pl->max_streams * 8));
  HIP_TRY(hipMalloc(&pl->d_sync, (size_t)pl->max_streams * 8));
  HIP_TRY(hipMalloc((void**)&pl->d_edge, (size_t)(pl->max_streams * 2 * (int64_t)pl->p.pad * 8)));
  return AMR_OK;
}

// Live-column layout for this plan (amr_internal.h LiveCols), or off: needs a
// two-pass length n = n1 * n2 with n1 a multiple of sps and a decision window.
// Every index the kernels use is checked here on the host (the float
// divisions of lc_div, the [L | D] offsets as a bijection onto [0, n)).
LiveCols plan_live_cols(const FftShape& f, const FskParams& p) {
  LiveCols lc{};
  static const bool off = [] { const char* e = std::getenv("AMR_FSK_LIVE"); return e && e[0] == '0'; }();
  const int64_t q = p.sps / 4, half = p.sps / 2;
  if (off || f.bluestein || f.six || p.n_bits == 0 || q < 1) return lc;
  const int n1 = f.n1, n2 = f.n2;
  if (p.sps > n1 || n1 % p.sps != 0 || (int64_t)n1 * n2 != p.n) return lc;
  lc.n1 = n1;
  lc.n2 = n2;
  lc.sps = (int)p.sps;
  lc.w0 = (int)(half - q);
  lc.nw = (int)(2 * q);
  lc.nl = n1 / lc.sps * lc.nw;
  lc.nd = n1 - lc.nl;
  lc.inv_n1 = 1.0f / (float)n1;
  lc.inv_sps = 1.0f / (float)lc.sps;
  lc.inv_nw = 1.0f / (float)lc.nw;
  lc.inv_ndp = 1.0f / (float)(lc.sps - lc.nw);
  if (lc.nd < 1) return LiveCols{};
  for (int j1 = 0; j1 < n1; ++j1) {
    bool live = false;
    const int pos = lc_col_pos(lc, j1, live);
    const int v = j1 % lc.sps;
    if (live != (v >= lc.w0 && v < lc.w0 + lc.nw)) return LiveCols{};
    if ((live ? lc_live_col(lc, pos) : lc_dead_col(lc, pos)) != j1) return LiveCols{};
  }
  std::vector<uint8_t> seen((size_t)p.n, 0);
  for (int64_t i = 0; i < p.n; ++i) {
    const int64_t o = lc_zoff(lc, (int)i);
    if (o < 0 || o >= p.n || seen[(size_t)o]) return LiveCols{};
    seen[(size_t)o] = 1;
  }
  lc.on = 1;
  static const bool no_prune = [] { const char* e = std::getenv("AMR_FFT_PRUNE"); return e && e[0] == '0'; }();
  lc.prune = !no_prune;
  return lc;
}

// Sizes of an FSK plan's device buffers from its shape alone (no device
// work): amr_fsk_plan_create allocates exactly these; amr_fsk_plan_bytes_estimate
// sums them for the drop-in plan cache before it creates a plan.
struct FskGeom {
  FskParams p{};
  FftShape sh;
  int64_t z = 0, u = 0, v = 0, dd = 0, cmp = 0, words = 0, six = 0, staging = 0, out = 0, out_cap = 0;
  int64_t split = 0;       // the split F1's buffers for up to kFskSplitMaxStreams streams (allocated on use)
  bool keep_z = false;
  bool dd_eager = false;   // AMR_FSK_KEEPZ=1: dd at creation (else on the first host entry)
  // the exact path: flags, scales, list, slots, exact bits, pocketfft tables
  bool exact = false;
  int n_slots = 0;
  int64_t slot_doubles = 0, xflags = 0, amb = 0, xlist = 0, xslots = 0, xbits = 0, xpool = 0, xplan = 0;
  int64_t total() const {
    return z + u + v + dd + cmp + words + six + staging + out + xflags + amb + xlist + xslots + xbits + xpool + xplan +
           split;
  }
};
bool fsk_geometry(int64_t n, int64_t sps, int nt, int64_t max_streams, FskGeom& g) {
  FskParams& p = g.p;
  p.n = n;
  p.sps = sps;
  p.nt = nt;
  p.pad = 3 * nt;
  const int64_t q = sps / 4, half = sps / 2;
  p.n_bits = (q > 0 && n > half) ? (n - half + sps - 1) / sps : 0;
  p.n_words = p.n_bits > 0 ? (p.n_bits + 31) / 32 : 1;
  g.out_cap = p.n_bits / 8 + 1;
  if (!fft_shape(n, g.sh)) return false;
  const int64_t M = g.sh.M;
  const bool plain = g.sh.bluestein || g.sh.six;   // epilogue in natural order (post kernel)
  p.rn1 = plain ? n : g.sh.n1;
  p.rn2 = plain ? 1 : g.sh.n2;
  p.lc = plan_live_cols(g.sh, p);
  p.bits_stride = p.lc.on ? (int64_t)((p.lc.nl + 7) >> 3) * p.rn2 : fft_bits_stride(p.rn1, p.rn2);
  p.inv_rn1 = 1.0f / (float)p.rn1;
  const int64_t s1_bytes = fsk_bandpass_scratch_bytes(max_streams, n, p.pad);
  if (p.lc.on) {
    // C: the live columns' transform; before the column pass it holds F1's checkpoints
    g.u = std::max(max_streams * (int64_t)p.lc.nl * p.lc.n2 * 16, s1_bytes);
  } else {
    g.u = std::max(max_streams * M * 16, s1_bytes);
    g.v = max_streams * M * 16;
  }
  g.staging = max_streams * n * 8;                   // d_x, allocated on the first host call
  // z; after F2, the exact path's rows ([ordinal][n] (f_mark, f_space))
  g.z = max_streams * n * 16;
  g.cmp = max_streams * p.bits_stride;
  g.words = max_streams * p.n_words * 4;
  g.six = g.sh.six ? 2 * max_streams * M * 16 : 0;
  g.out = max_streams * (g.out_cap + 16 + 2 * (int64_t)p.pad * 8);   // host-API output staging + edge table
  // (+ FS0's tables, w <= n / 4, and start states at L >= kFskSplitConvMinL)
  // (+ the strict margin's per-tone scratch: 5 blocks rows of ceil(m1 / 16) and
  // two chunk rows, the maxima, and the tables -- W, K12, HS, TZ <= 4 w / 16 + 64 each)
  const int64_t m1g = n + 2 * (int64_t)p.pad;
  const int64_t strict_row = 5 * ((m1g + kStrictBlk - 1) / kStrictBlk) + 2 * (m1g / kFskSplitConvMinL + 2);
  g.split = std::min<int64_t>(max_streams, kFskSplitMaxStreams) *
                (2 * m1g * 8 + 8 + 96 * (m1g / kFskSplitConvMinL + 2) + 2 * (strict_row * 8 + 64)) +
            2 * (2 * (n / 4) + 1) * 48 + 2 * (2 * (n / 4) + 1 + 4 * (2 * (n / 4) / 16 + 64) + 64) * 8;
  // the exact path (AMR_FSK_EXACT=0: off), at every length with decisions to make
  static const bool exact_env = [] { const char* e = std::getenv("AMR_FSK_EXACT"); return !(e && e[0] == '0'); }();
  g.exact = exact_env && p.n_bits > 0;
  if (g.exact) {
    g.slot_doubles = pf_even(n) + pf_scratch_doubles_n(n);   // the row, then its transforms' scratch
    // one persistent workgroup per slot: up to 2 per stream and 512 (2 per
    // CU; the launch takes no more than are resident at once, E2's register
    // budget allows one per CU), within 2 GiB of slots
    g.n_slots = (int)std::max<int64_t>(
        1, std::min<int64_t>({2 * max_streams, 512, ((int64_t)1 << 31) / (g.slot_doubles * 8)}));
    g.xflags = (max_streams + 31) / 32 * 4;
    g.amb = max_streams * 8;
    g.xlist = (max_streams + 1) * 4;
    g.xslots = (int64_t)g.n_slots * g.slot_doubles * 8;
    g.xbits = max_streams * p.bits_stride;
    g.xpool = pf_pool_doubles_bound(n) * 8;
    g.xplan = (int64_t)sizeof(PfLen);
    // live layout: keep all of z through F2 (the exact path then needs no F1
    // re-run); the dead tiles' transform and the staged input go to dd
    // (AMR_FSK_KEEPZ=0, an A/B switch: dead tiles in place, the F1 re-run)
    // (AMR_FSK_F1_FMA=1 makes F1 the contracted form, not scipy's order: the
    // exact path must then re-run F1 in scipy's order, so no keep_z)
    static const bool keepz_env = [] {
      const char* e = std::getenv("AMR_FSK_KEEPZ");
      const char* f = std::getenv("AMR_FSK_F1_FMA");
      return !(e && e[0] == '0') && !(f && f[0] == '1');
    }();
    static const bool eager_env = [] { const char* e = std::getenv("AMR_FSK_KEEPZ"); return e && e[0] == '1'; }();
    g.keep_z = keepz_env && p.lc.on && (int64_t)p.lc.nd * p.lc.n2 * 2 >= n;
    if (g.keep_z) {
      g.dd = max_streams * (int64_t)p.lc.nd * p.lc.n2 * 16;   // counted: a host entry allocates it
      g.dd_eager = eager_env;
      g.staging = 0;
    }
  }
  return true;
}

// The split F1's design (the PSK layout's rule, iir_design.h):
// per tone, a chunk's outputs differ from scipy's by (1) the zero start,
// decayed after w samples to tail(w) * zmax * 3 peak (the odd extension
// triples the input peak) and carried through the backward pass (its L1 gain
// h1) -- w is chosen to bring that below u G / 16 -- and (2) a different
// rounding trajectory, G = g1 (1 + h1): the forward pass's rounding (noise
// gain g1) filtered backward, plus the backward pass's own.  kappa = 64.25 u
// G over the tones (measured >= 30x above the worst error,
// tests/test_split_margin.py); an envelope then moves by at most kappa *
// ||ifft(h)||_1 * peak|ext x|, the margin F2 adds for split calls.  Refused
// when a warm-up exceeds n / 4 or the margin would pass 2^-24 of the peak.
constexpr double kFskSplitSafety = 64.0;
bool fsk_split_design(const FskIir& f, int nt, int64_t n, int64_t* w_out, double* kappa_out, double* hl1_out) {
  if (nt != 7 || n < 64) return false;
  const double u = 0x1p-53;
  IirGains g[2];
  double G = 0.0;
  for (int t = 0; t < 2; ++t) {
    Iir fi{};
    fi.nt = nt;
    for (int i = 0; i < nt; ++i) {
      fi.b[i] = f.b[t][i];
      fi.a[i] = f.a[t][i];
    }
    g[t] = iir_gains(fi);
    if (!g[t].ok) return false;
    G = std::max(G, g[t].g1 * (1.0 + g[t].h1));
  }
  const double tol = 0x1p-4 * u * G;
  int64_t w = 0;
  for (int t = 0; t < 2; ++t) {
    const int64_t wt = warmup_for(g[t], g[t].zmax * 3.0 * g[t].h1, tol);
    if (wt < 0) return false;
    w = std::max(w, wt);
  }
  const double kappa = (kFskSplitSafety + 0.25) * u * G;
  const double hl1 = hilbert_l1(n) * (1.0 + 0x1p-20);
  if (w > n / 4 || !(kappa * hl1 <= 0x1p-16)) return false;
  *w_out = w;
  *kappa_out = kappa;
  *hl1_out = hl1;
  return true;
}

// F2's margin scale tau from a standard FFT rounding bound (round 6, DESIGN.md
// §2 item 6).  F2 keeps a compare only when |env_mark - env_space| > 2 tau
// peak|ext x|; the fast path's and pocketfft's envelopes each differ from
// |hilbert(z)| in exact arithmetic by at most (4 eps + 4u) ||z||_2 per tone,
// eps the transform's relative 2-norm error:
//   direct (FFTPACK-style / two-pass / six-step) length M, widest radix p:
//     eps = L eta / (1 - L eta), L = ceil(log2 M), eta = max(8.5u, sqrt(p)
//     gamma_{p+4} / log2 p) + 2u (a radix-p pass's 2-norm error per binary
//     level -- Higham's radix-2 eta = mu + gamma_4 (sqrt2 + mu) generalised --
//     plus twiddles within 2u);
//   Bluestein (n, M): (Bmax / sqrt n) (2 eps_M + 2 gc) + sqrt(2n - 1) eps_M +
//     gc, gc = sqrt2 gamma_2 + 2u (a complex product with a rounded chirp):
//     the chirp product, FFT_M, the product with the kernel's spectrum (whose
//     own FFT-computed table is off by <= eps_M ||B||_2 = eps_M sqrt(M (2n -
//     1)) -- the sqrt(2n - 1) term), IFFT_M, the chirp product.  Bmax =
//     max |FFT_M(kernel)| <= sqrt(n) (6 + 2 ln n): the chirp exp(i pi m^2 / n)
//     is periodic (n or 2n) with Fourier coefficients of modulus 1 / sqrt(n)
//     (a quadratic Gauss sum), so the windowed kernel's spectrum is a sum of
//     Dirichlet kernels D_{2n-1}, whose values on a grid sum to <= 2 (2n - 1)
//     + P (ln(P / 2) + 1) (measured max |B| = 2.0-2.2 sqrt(n));
// and ||z||_2 <= (G^2 sqrt(m1) + 2 G R + R^2) peak|ext x| per tone (G the
// band-pass's L1 gain, R the L2 norm of its zi-start transient: both
// filtfilt passes).  tau = max(2^-36, (4 eps_fast + 4 eps_ref + 8u) max
// ||z||_2 / peak): a compare F2 keeps cannot differ between the two paths.
// ~13 x 2^-36 at n = 96000 (the measured difference stays ~1e-15 of the
// peak, tests/test_gpu_fsk.py); the flag rate of real signals is unchanged.
struct FskFftBound {
  double tau = 0.0, eps_fast = 0.0, eps_ref = 0.0, zmax = 0.0;
  bool fast_blue = false, ref_blue = false;
  int64_t fast_M = 0, ref_M = 0;
};
int64_t lpf_of(int64_t n) {
  int64_t r = 1;
  for (int64_t q = 2; q * q <= n; ++q)
    while (n % q == 0) {
      r = q;
      n /= q;
    }
  return n > 1 ? std::max(r, n) : r;
}
bool fsk_fft_bound(const FskIir& f, int nt, int64_t n, int pad, FskFftBound& o) {
  const double u = 0x1p-53;
  auto gam = [&](double k) { return k * u / (1.0 - k * u); };
  auto eta_of = [&](int64_t p) {
    const double r = (double)std::max<int64_t>(p, 2);
    return std::max(8.5 * u, std::sqrt(r) * gam(r + 4.0) / std::max(1.0, std::log2(r))) + 2.0 * u;
  };
  auto eps_direct = [&](int64_t M, int64_t p) {
    const double e = std::ceil(std::log2((double)std::max<int64_t>(M, 2))) * eta_of(p);
    return e / (1.0 - e);
  };
  const double gc = std::sqrt(2.0) * gam(2.0) + 2.0 * u;
  const double bq = 6.0 + 2.0 * std::log((double)n);   // Bmax / sqrt(n)
  auto eps_blue = [&](int64_t M) {
    const double em = eps_direct(M, lpf_of(M));
    return bq * (2.0 * em + 2.0 * gc) + std::sqrt(2.0 * (double)n - 1.0) * em + gc;
  };
  FftShape sh;
  if (!fft_shape(n, sh)) return false;
  bool rb = false;
  int64_t rn2 = n, rp = 1;
  pf_hilbert_shape(n, &rb, &rn2, &rp);
  o.fast_blue = sh.bluestein;
  o.fast_M = sh.M;
  o.ref_blue = rb;
  o.ref_M = rn2;
  o.eps_fast = sh.bluestein ? eps_blue(sh.M) : eps_direct(n, lpf_of(n));
  o.eps_ref = rb ? eps_blue(rn2) : eps_direct(n, rp);
  const double m1 = (double)(n + 2 * (int64_t)pad);
  double zb = 0.0;
  for (int t = 0; t < 2; ++t) {
    Iir fi{};
    fi.nt = nt;
    for (int i = 0; i < nt; ++i) {
      fi.b[i] = f.b[t][i];
      fi.a[i] = f.a[t][i];
    }
    for (int i = 0; i < nt - 1; ++i) fi.zi[i] = f.zi[t][i];
    const IirGains g = iir_gains(fi);
    const double R = zi_response_l2(fi);
    if (!g.ok || !(R >= 0.0)) return false;
    const double G = g.h1 * (1.0 + 0x1p-20);
    zb = std::max(zb, G * G * std::sqrt(m1) + 2.0 * G * R + R * R);
  }
  o.zmax = zb;
  const double tau = (4.0 * o.eps_fast + 4.0 * o.eps_ref + 8.0 * u) * zb * (1.0 + 0x1p-20);
  o.tau = std::max(kAmbTau, tau);
  return std::isfinite(o.tau);
}

}  // namespace

extern "C" {

int amr_fsk_fft_margin(int64_t n, const double* mb, const double* ma, const double* mzi, const double* sb,
                       const double* sa, const double* szi, int nt, double* out) {
  if (!mb || !ma || !mzi || !sb || !sa || !szi || !out || nt < 2 || nt > 8 || n <= 3 * nt)
    return fail(AMR_E_INVALID, "amr_fsk_fft_margin: bad argument");
  FskIir f{};
  for (int i = 0; i < nt; ++i) {
    f.b[0][i] = mb[i];
    f.a[0][i] = ma[i];
    f.b[1][i] = sb[i];
    f.a[1][i] = sa[i];
  }
  for (int i = 0; i < nt - 1; ++i) {
    f.zi[0][i] = mzi[i];
    f.zi[1][i] = szi[i];
  }
  FskFftBound o;
  if (!fsk_fft_bound(f, nt, n, 3 * nt, o)) return fail(AMR_E_INVALID, "amr_fsk_fft_margin: no bound for these filters at n");
  out[0] = o.tau;
  out[1] = o.eps_fast;
  out[2] = o.eps_ref;
  out[3] = o.zmax;
  out[4] = o.fast_blue ? 1.0 : 0.0;
  out[5] = (double)o.fast_M;
  out[6] = o.ref_blue ? 1.0 : 0.0;
  out[7] = (double)o.ref_M;
  return AMR_OK;
}

int amr_fsk_plan_margin(amr_fsk_plan* plan, double* tau, double* tau_split) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  if (tau) *tau = plan->p.tau;
  if (tau_split) *tau_split = plan->split_tau;
  return AMR_OK;
}

int amr_fsk_split_design(int64_t n, const double* mb, const double* ma, const double* sb, const double* sa, int nt,
                         int64_t* warmup, double* kappa, double* hilbert_l1_out) {
  if (!mb || !ma || !sb || !sa || nt != 7) return fail(AMR_E_INVALID, "amr_fsk_split_design: bad argument");
  FskIir f{};
  for (int i = 0; i < nt; ++i) {
    f.b[0][i] = mb[i];
    f.a[0][i] = ma[i];
    f.b[1][i] = sb[i];
    f.a[1][i] = sa[i];
  }
  int64_t w = 0;
  double k = 0.0, h = 0.0;
  if (!fsk_split_design(f, nt, n, &w, &k, &h)) return fail(AMR_E_INVALID, "no time-split design for these filters at n");
  if (warmup) *warmup = w;
  if (kappa) *kappa = k;
  if (hilbert_l1_out) *hilbert_l1_out = h;
  return AMR_OK;
}

int64_t amr_fsk_plan_bytes_estimate(int64_t n, int64_t sps, int ntaps, int64_t max_streams) {
  if (n < 1 || sps < 1 || ntaps < 1 || max_streams < 1)
    return fail(AMR_E_INVALID, "amr_fsk_plan_bytes_estimate: bad argument");
  FskGeom g;
  if (!fsk_geometry(n, sps, ntaps, max_streams, g)) return fail(AMR_E_INVALID, "no FFT plan for this length");
  return g.total();
}

int amr_fsk_plan_create(amr_fsk_plan** out, int device, int64_t n, int64_t sps, const double* mb, const double* ma,
                        const double* mzi, const double* sb, const double* sa, const double* szi, int nt,
                        int64_t max_streams) {
  if (!out || !mb || !ma || !mzi || !sb || !sa || !szi) return fail(AMR_E_INVALID, "amr_fsk_plan_create: NULL argument");
  *out = nullptr;
  if (sps < 1 || max_streams < 1) return fail(AMR_E_INVALID, "bad sps/max_streams");
  if (nt != 7) return fail(AMR_E_INVALID, "FSK band-pass must have 7 taps (butter(3, band))");
  if (ma[0] != 1.0 || sa[0] != 1.0) return fail(AMR_E_INVALID, "a[0] must be 1 (scipy butter form)");
  if (n <= 3 * nt)
    return fail(AMR_E_PADLEN, "The length of the input vector x must be greater than padlen, which is " +
                                  std::to_string(3 * nt) + ".");
  auto* pl = new amr_fsk_plan();
  pl->device = device;
  hipError_t e = hipSetDevice(device);
  if (e != hipSuccess) {
    delete pl;
    return fail(AMR_E_NODEVICE, std::string("hipSetDevice: ") + hipGetErrorString(e));
  }
  FskGeom geo;
  if (!fsk_geometry(n, sps, nt, max_streams, geo)) {
    delete pl;
    return fail(AMR_E_INVALID, "no FFT plan for length " + std::to_string(n));
  }
  FskParams& p = pl->p;
  p = geo.p;
  for (int i = 0; i < nt; ++i) {
    pl->f.b[0][i] = mb[i];
    pl->f.a[0][i] = ma[i];
    pl->f.b[1][i] = sb[i];
    pl->f.a[1][i] = sa[i];
  }
  for (int i = 0; i < nt - 1; ++i) {
    pl->f.zi[0][i] = mzi[i];
    pl->f.zi[1][i] = szi[i];
  }
  pl->max_streams = max_streams;
  pl->out_cap = geo.out_cap;
  e = hipStreamCreateWithFlags(&pl->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    fsk_plan_free(pl);
    return fail(AMR_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  if (int rc = fft_plan_init(pl->fft, n, pl->stream, max_streams)) {
    fsk_plan_free(pl);
    return rc;
  }
  if (pl->fft.six) pl->scratch_bytes += geo.six;
  pl->u_bytes = geo.u;
  pl->staging_bytes = geo.staging;
  pl->dd_bytes = geo.dd;
  pl->split_reserved = geo.split;
  struct A { void** ptr; int64_t bytes; };
  const A allocs[] = {
      {(void**)&pl->z, geo.z},
      {(void**)&pl->u, geo.u},
      {(void**)&pl->v, geo.v},
      {(void**)&pl->dd, geo.dd_eager ? geo.dd : 0},
      {(void**)&pl->cmp, geo.cmp},
      {(void**)&pl->words, geo.words},
      {(void**)&pl->xflags, geo.xflags},
      {(void**)&pl->amb, geo.amb},
      {(void**)&pl->xlist, geo.xlist},
      {(void**)&pl->xslots, geo.xslots},
      {(void**)&pl->xbits, geo.xbits},
      {(void**)&pl->xpool, geo.xpool},
      {(void**)&pl->xL, geo.xplan},
  };
  for (const A& a : allocs) {
    if (a.bytes == 0) continue;
    e = hipMalloc(a.ptr, (size_t)a.bytes);
    if (e != hipSuccess) {
      fsk_plan_free(pl);
      return fail(AMR_E_NOMEM, "hipMalloc(" + std::to_string(a.bytes) + " B): " + hipGetErrorString(e));
    }
    pl->scratch_bytes += a.bytes;
  }
  if (geo.exact) {
    // E2's grid hint (FskExact count_hint): none yet, so the full grid
    e = hipHostMalloc((void**)&pl->xcount_host, sizeof(int32_t), hipHostMallocMapped);
    if (e == hipSuccess) {
      *pl->xcount_host = (int32_t)max_streams;
      for (int32_t& h : pl->hint_hist) h = (int32_t)max_streams;
      e = hipHostGetDevicePointer((void**)&pl->xcount_dev, pl->xcount_host, 0);
    }
    if (e != hipSuccess) {
      fsk_plan_free(pl);
      return fail(AMR_E_NOMEM, std::string("hipHostMalloc (exact-path count hint): ") + hipGetErrorString(e));
    }
    // pocketfft's plans of length n: tables to the device, then the Bluestein
    // tables that need a device transform (into the envelope slots' scratch)
    std::vector<double> pool;
    PfLen L{};
    if (!pf_len_build(n, L, pool) || (int64_t)pool.size() > geo.xpool / 8 || geo.xslots / 8 < 4 * L.bl.n2) {
      fsk_plan_free(pl);
      return fail(AMR_E_INVALID, "exact path: pocketfft plan of length " + std::to_string(n));
    }
    e = hipMemcpy(pl->xpool, pool.data(), pool.size() * 8, hipMemcpyHostToDevice);
    if (e == hipSuccess) e = hipMemcpy(pl->xL, &L, sizeof(PfLen), hipMemcpyHostToDevice);
    if (e == hipSuccess) e = pf_finish(L, pl->xL, pl->xpool, pl->xslots, pl->stream);
    if (e == hipSuccess) e = hipMemset(pl->xflags, 0, (size_t)geo.xflags);
    if (e != hipSuccess) {
      fsk_plan_free(pl);
      return fail(AMR_E_HIP, std::string("exact path tables: ") + hipGetErrorString(e));
    }
    pl->exact_on = true;
    pl->x_lean = pf_hilbert_lean(L);
    // keep_z reads z in the [L | D] layout through the lean kernel only; a
    // live-layout length is 5-smooth, so pocketfft's plans are always lean
    pl->keep_z = geo.keep_z;
    if (pl->keep_z && !pl->x_lean) {
      fsk_plan_free(pl);
      return fail(AMR_E_INVALID, "exact path: live-layout length " + std::to_string(n) + " without a lean plan");
    }
    pl->p.amb = pl->amb;
    pl->p.xflags = pl->xflags;         // F3 reads a flagged stream's bits from xbits
    pl->p.xbits = pl->xbits;
    pl->n_slots = geo.n_slots;
    pl->slot_doubles = geo.slot_doubles;
    static const bool xstream_on = [] { const char* e = std::getenv("AMR_FSK_XSTREAM"); return e && e[0] == '1'; }();
    if (xstream_on) {
      int least = 0, greatest = 0;
      e = hipDeviceGetStreamPriorityRange(&least, &greatest);
      if (e == hipSuccess) e = hipStreamCreateWithPriority(&pl->xstream, hipStreamNonBlocking, greatest);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&pl->ev_f2, hipEventDisableTiming);
      if (e == hipSuccess) e = hipEventCreateWithFlags(&pl->ev_x, hipEventDisableTiming);
      if (e != hipSuccess) {
        fsk_plan_free(pl);
        return fail(AMR_E_HIP, std::string("exact-path stream: ") + hipGetErrorString(e));
      }
    }
  }
  {
    FskFftBound fb;
    if (!fsk_fft_bound(pl->f, nt, n, p.pad, fb)) {
      fsk_plan_free(pl);
      return fail(AMR_E_INVALID, "no FFT rounding bound for these filters at length " + std::to_string(n));
    }
    p.tau = fb.tau;
    double kappa = 0.0, hl1 = 0.0;
    pl->split_ok = fsk_split_design(pl->f, nt, n, &pl->split_w, &kappa, &hl1);
    pl->split_kappa = kappa;
    pl->split_hl1 = hl1;
    pl->split_tau = p.tau + kappa * hl1;
    if (pl->split_ok) {   // FS0's tables, per tone: K [w][6], then Z0 [w + 1][6]
      const int64_t w = pl->split_w;
      pl->split_tab_host.assign((size_t)(2 * w + 2 * (w + 1)) * 6, 0.0);
      for (int t = 0; t < 2; ++t) {
        Iir fi{};
        fi.nt = nt;
        for (int i = 0; i < nt; ++i) { fi.b[i] = pl->f.b[t][i]; fi.a[i] = pl->f.a[t][i]; fi.zi[i] = pl->f.zi[t][i]; }
        split_state_tables(fi, w, pl->split_tab_host.data() + (size_t)t * w * 6,
                           pl->split_tab_host.data() + (size_t)(2 * w + t * (w + 1)) * 6);
      }
    }
  }
  *out = pl;
  return AMR_OK;
}

int amr_fsk_plan_destroy(amr_fsk_plan* plan) {
  fsk_plan_free(plan);
  return AMR_OK;
}
int64_t amr_fsk_plan_out_capacity(const amr_fsk_plan* plan) { return plan ? plan->out_cap : -1; }
int64_t amr_fsk_plan_scratch_bytes(const amr_fsk_plan* plan) {
  if (!plan) return -1;
  // scratch + the host-API staging (allocated on the first amr_fsk_demod_host:
  // d_x, or dd on a plan that keeps z)
  return plan->scratch_bytes + plan->staging_bytes + (plan->dd ? 0 : plan->dd_bytes) +
         plan->max_streams * (plan->out_cap + 16 + 2 * (int64_t)plan->p.pad * 8) +
         std::max(plan->split_reserved, plan->split_alloc + plan->strict_bytes);   // == fsk_geometry().total() (split calls <= 1024 streams)
}
int64_t amr_fsk_plan_resident_bytes(const amr_fsk_plan* plan) {
  if (!plan) return -1;
  // what is allocated now: a plan that only ever ran the device entry holds
  // no staging (no d_x, no dd, no output staging)
  return plan->scratch_bytes + (plan->d_x ? plan->staging_bytes : 0) +
         (plan->d_out ? plan->max_streams * (plan->out_cap + 16 + 2 * (int64_t)plan->p.pad * 8) : 0) +
         plan->split_alloc + plan->strict_bytes;
}
int64_t amr_fsk_plan_fft_length(const amr_fsk_plan* plan) { return plan ? plan->fft.M : -1; }
int amr_fsk_plan_live_columns(const amr_fsk_plan* plan) { return plan ? plan->p.lc.on : -1; }

int amr_fsk_plan_split_conv(amr_fsk_plan* plan) {
  if (!plan) return -1;
  std::lock_guard<std::mutex> lk(plan->mu);
  return fsk_split_conv_on(plan) ? 1 : 0;
}

int amr_fsk_plan_set_layout(amr_fsk_plan* plan, int layout) {
  if (!plan || layout < AMR_FSK_LAYOUT_AUTO || layout > AMR_FSK_LAYOUT_SPLIT)
    return fail(AMR_E_INVALID, "amr_fsk_plan_set_layout: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  plan->split_mode = layout;
  return AMR_OK;
}

int amr_fsk_plan_split_info(amr_fsk_plan* plan, int* last_split, int64_t* warmup, int64_t* chunk, double* kappa,
                            double* tau) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);   // run_fsk / fsk_split_params write these under it
  if (last_split) *last_split = plan->last_split ? 1 : 0;
  if (warmup) *warmup = plan->split_ok ? plan->split_w : -1;
  if (chunk) *chunk = plan->split_L;
  if (kappa) *kappa = plan->split_kappa;
  if (tau) *tau = plan->split_tau;
  return AMR_OK;
}

int amr_fsk_plan_set_split_strict(amr_fsk_plan* plan, int mode) {
  if (!plan || mode < -1 || mode > 1) return fail(AMR_E_INVALID, "amr_fsk_plan_set_split_strict: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  plan->strict_mode = mode;
  return AMR_OK;
}

int amr_fsk_plan_split_strict(amr_fsk_plan* plan) {
  if (!plan) return -1;
  std::lock_guard<std::mutex> lk(plan->mu);
  return fsk_split_strict_on(plan) ? 1 : 0;
}

int amr_fsk_plan_last_strict(amr_fsk_plan* plan) {
  if (!plan) return -1;
  std::lock_guard<std::mutex> lk(plan->mu);
  return plan->last_strict ? 1 : 0;
}

int amr_fsk_split_strict_design(const double* b, const double* a, const double* zi, int nt, int64_t w, double* consts,
                                double* tabs) {
  if (!b || !a || !zi || !consts || nt < 2 || nt > kMaxTaps || w < 1)
    return fail(AMR_E_INVALID, "amr_fsk_split_strict_design: bad argument");
  Iir f{};
  f.nt = nt;
  for (int i = 0; i < nt; ++i) { f.b[i] = b[i]; f.a[i] = a[i]; }
  for (int i = 0; i < nt - 1; ++i) f.zi[i] = zi[i];
  const int N = nt - 1;
  std::vector<double> tab((size_t)(2 * w + 1) * N);
  split_state_tables(f, w, tab.data(), tab.data() + (size_t)w * N);
  StrictDesign d;
  const bool ok = strict_design_bp(f, tab.data(), tab.data() + (size_t)w * N, w, d, strict_detail::responses(f)) &&
                  d.g1x * (d.kx + 2.0 * d.ky) < 0.125;
  // the PSK entry's layout (amr_psk_split_strict_design) without the low-pass
  const double v[32] = {d.g1x, d.gmax, d.hz, d.tk, d.zi_sum, d.zb, d.kx, d.ky, 2.0 * 0x1p-53 * (1.0 + 0x1p-50),
                        d.gam, 0.0, (double)w, 0.0, 0.0, (double)d.W.size(), (double)d.K12.size(),
                        (double)d.HS.size(), (double)d.GS.size(), (double)d.TZ.size(), (double)d.k12_off, d.w_tail,
                        d.k12_tail, d.hs_tail, d.tz_tail, 0.0, 0.0, ok ? 1.0 : 0.0, 0.0};
  for (int i = 0; i < 32; ++i) consts[i] = v[i];
  if (!ok) return fail(AMR_E_INVALID, "no strict bound for this filter");
  if (tabs) {
    double* o = tabs;
    for (const std::vector<double>* t : {&d.kabs, &d.z0abs, &d.W, &d.K12, &d.HS, &d.GS, &d.TZ}) {
      std::memcpy(o, t->data(), t->size() * 8);
      o += t->size();
    }
  }
  return AMR_OK;
}

int amr_fsk_split_bounds_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                              double* z_out, double* bnd_out, double* peak_out) {
  if (!plan || !x || !z_out || !bnd_out || !peak_out || B < 1)
    return fail(AMR_E_INVALID, "amr_fsk_split_bounds_host: bad argument");
  if (!dtype_size(dtype)) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (!plan->split_ok || !fsk_split_conv_on(plan)) return fail(AMR_E_INVALID, "no convolution-start split F1 for this plan");
  if (B > plan->max_streams || B > 65535) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  const int saved = plan->strict_mode;
  plan->strict_mode = 1;
  int rc = fsk_strict_prepare(plan);
  if (!rc && !plan->strict_ok) rc = fail(AMR_E_INVALID, "no strict bound for this plan's filters");
  const int64_t n = plan->p.n;
  void* xs = nullptr;
  if (!rc) rc = stage_input(plan, x, dtype, B, x_stride, &xs);
  if (!rc) rc = ensure_split_buffers(plan, B);
  FskParams p = plan->p;
  p.lc = LiveCols{};                         // natural order for the caller
  p.amb = nullptr;
  FskSplit sp{};
  if (!rc) {
    sp = fsk_split_params(plan, B, 0);
    rc = ensure_split_conv(plan, sp, B);
  }
  if (!rc) rc = ensure_fsk_strict(plan, sp, B);
  if (!rc && !sp.strict) rc = fail(AMR_E_INVALID, "no strict bound for this call's chunk (not a multiple of 16)");
  plan->strict_mode = saved;
  if (rc) return rc;
  HIP_TRY(launch_fsk_split(dtype, xs, n, B, plan->z, p, plan->f, sp, plan->stream));
  HIP_TRY(hipMemcpyAsync(z_out, plan->z, (size_t)(B * n * 16), hipMemcpyDeviceToHost, plan->stream));
  std::vector<unsigned long long> hb((size_t)B * 16), hp((size_t)B);
  HIP_TRY(hipMemcpyAsync(hb.data(), sp.bnd, hb.size() * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipMemcpyAsync(hp.data(), sp.peak, hp.size() * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  std::memcpy(bnd_out, hb.data(), hb.size() * 8);
  std::memcpy(peak_out, hp.data(), hp.size() * 8);
  return AMR_OK;
}

int amr_fsk_split_bandpass_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                                int64_t chunk, double* out) {
  if (!plan || (B && (!x || !out))) return fail(AMR_E_INVALID, "amr_fsk_split_bandpass_host: NULL argument");
  if (!dtype_size(dtype)) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (!plan->split_ok) return fail(AMR_E_INVALID, "the plan's filters have no time-split design");
  if (B > plan->max_streams || B > 65535) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  // FS0's start states are B x 2 x ceil(m1 / L) x 48 B (outside split_reserved's
  // L >= kFskSplitConvMinL estimate): a smaller chunk is refused
  if (chunk < 0 || (chunk > 0 && chunk < kFskSplitConvMinL && fsk_split_conv_on(plan)))
    return fail(AMR_E_INVALID, "amr_fsk_split_bandpass_host: chunk must be 0 (the plan's) or >= 128 with the convolution starts");
  if (B == 0) return AMR_OK;
  const int64_t n = plan->p.n;
  void* xs = nullptr;
  if (int rc = stage_input(plan, x, dtype, B, x_stride, &xs)) return rc;
  if (int rc = ensure_split_buffers(plan, B)) return rc;
  FskParams p = plan->p;
  p.lc = LiveCols{};                         // natural order for the caller
  p.amb = nullptr;
  FskSplit sp = fsk_split_params(plan, B, chunk);
  if (int rc = ensure_split_conv(plan, sp, B)) return rc;
  HIP_TRY(launch_fsk_split(dtype, xs, n, B, plan->z, p, plan->f, sp, plan->stream));
  HIP_TRY(hipMemcpyAsync(out, plan->z, (size_t)(B * n * 16), hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  return AMR_OK;
}

int amr_fsk_plan_synchronize(amr_fsk_plan* plan) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  HIP_TRY(gate_sync(plan->gate));
  return AMR_OK;
}

int amr_fsk_plan_enable_timing(amr_fsk_plan* plan, int on) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (on && !plan->ev[0][0]) {
    for (auto& e : plan->ev)
      for (auto& h : e) HIP_TRY(hipEventCreate(&h));
  }
  plan->timing = on != 0;
  return AMR_OK;
}

int amr_fsk_plan_set_exact_mode(amr_fsk_plan* plan, int mode) {
  if (!plan || mode < 0 || mode > 2) return fail(AMR_E_INVALID, "amr_fsk_plan_set_exact_mode: bad argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  if (mode != 0 && !plan->exact_on) return fail(AMR_E_INVALID, "this plan has no exact path (no decisions, or AMR_FSK_EXACT=0)");
  plan->exact_mode = mode;
  // F3 reads a flagged stream's bits from xbits only while the exact path runs
  plan->p.xflags = mode ? plan->xflags : nullptr;
  return AMR_OK;
}

int amr_fsk_plan_exact_streams(amr_fsk_plan* plan, int64_t* count) {
  if (!plan || !count) return fail(AMR_E_INVALID, "NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  *count = 0;
  if (!plan->exact_on || !plan->ran_exact) return AMR_OK;
  int32_t c = 0;
  HIP_TRY(hipMemcpy(&c, plan->xlist + plan->max_streams, 4, hipMemcpyDeviceToHost));
  *count = c;
  return AMR_OK;
}

int amr_fsk_plan_timings(amr_fsk_plan* plan, float* ms, int count) {
  if (!plan || !ms) return fail(AMR_E_INVALID, "NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  for (int i = 0; i < count && i < AMR_TF_COUNT; ++i) {
    ms[i] = -1.0f;
    if (!plan->timing || !plan->ev_used[i]) continue;
    HIP_TRY(hipEventSynchronize(plan->ev[i][1]));   // the launch slot may end on a comm stream (a gather)
    HIP_TRY(hipEventElapsedTime(&ms[i], plan->ev[i][0], plan->ev[i][1]));
  }
  return AMR_OK;
}

int amr_fsk_allgather(amr_comm* comm, const void* d_send, void* d_recv, int64_t bytes_per_rank, amr_fsk_plan* plan) {
  if (!plan) return allgather_after(comm, d_send, d_recv, bytes_per_rank, nullptr, nullptr);
  std::lock_guard<std::mutex> lk(plan->mu);
  return allgather_after(comm, d_send, d_recv, bytes_per_rank, plan->stream, &plan->gate,
                         plan->timing && plan->ev_used[AMR_TF_LAUNCH] ? plan->ev[AMR_TF_LAUNCH][1] : nullptr);
}

int amr_fsk_demod_device(amr_fsk_plan* plan, const void* d_x, int dtype, int64_t n_streams, int64_t x_stride,
                         uint8_t* d_out, int64_t out_stride, int64_t* d_out_len, int64_t* d_sync_idx) {
  if (!plan || (n_streams && (!d_x || !d_out || !d_out_len || !d_sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_device: NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_fsk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx);
}

int amr_fsk_demod_device_edges(amr_fsk_plan* plan, const void* d_x, int dtype, int64_t n_streams, int64_t x_stride,
                               const double* d_edges, uint8_t* d_out, int64_t out_stride, int64_t* d_out_len,
                               int64_t* d_sync_idx) {
  if (!plan || (n_streams && (!d_x || !d_edges || !d_out || !d_out_len || !d_sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_device_edges: NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_fsk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx, d_edges);
}

}  // extern "C"

namespace {
int fsk_demod_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride, const double* edges,
                   uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  if (!plan || (B && (!x || !out || !out_len || !sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_host: NULL argument");
  if (!dtype_size(dtype)) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < plan->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  if (B == 0) return AMR_OK;
  const int64_t cap = plan->out_cap;
  if (int rc = ensure_out_staging(plan)) return rc;
  for (bool& u : plan->ev_used) u = false;
  if (plan->p.n_bits == 0) {
    if (int rc = fsk_empty_outputs(plan, B, plan->d_len, plan->d_sync)) return rc;
  } else {
    void* xs = nullptr;
    if (int rc = stage_input(plan, x, dtype, B, x_stride, &xs)) return rc;
    const double* d_edge = nullptr;
    if (edges) {
      HIP_TRY(hipMemcpyAsync(plan->d_edge, edges, (size_t)(B * 2 * (int64_t)plan->p.pad * 8), hipMemcpyHostToDevice,
                             plan->stream));
      d_edge = plan->d_edge;
    }
    plan->count_sync = true;                 // this call waits anyway: the exact path sized by its own count
    const int rc = run_fsk(plan, xs, dtype, B, plan->p.n, plan->d_out, cap, plan->d_len, plan->d_sync, d_edge);
    plan->count_sync = false;
    if (rc) return rc;
  }
  if (int rc = copy_batch_d2h(out, out_stride, plan->d_out, cap, out_stride < cap ? out_stride : cap, B,
                              plan->stream))
    return rc;
  HIP_TRY(hipMemcpyAsync(out_len, plan->d_len, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipMemcpyAsync(sync_idx, plan->d_sync, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  return AMR_OK;
}
}  // namespace

extern "C" {

int amr_fsk_demod_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride, uint8_t* out,
                       int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  return fsk_demod_host(plan, x, dtype, B, x_stride, nullptr, out, out_stride, out_len, sync_idx);
}

int amr_fsk_demod_host_edges(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                             const double* edges, uint8_t* out, int64_t out_stride, int64_t* out_len,
                             int64_t* sync_idx) {
  if (B && !edges) return fail(AMR_E_INVALID, "amr_fsk_demod_host_edges: NULL edges");
  return fsk_demod_host(plan, x, dtype, B, x_stride, edges, out, out_stride, out_len, sync_idx);
}

// Queued host entry (as amr_psk_demod_host_async): upload, demod, download on
// the plan's stream, no wait; host buffers untouched until amr_fsk_plan_synchronize.
int amr_fsk_demod_host_async(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                             uint8_t* out, int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  if (!plan || (B && (!x || !out || !out_len || !sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_host_async: NULL argument");
  const int64_t es = dtype_size(dtype);
  if (!es) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < plan->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  if (B == 0) return AMR_OK;
  const int64_t n = plan->p.n;
  const int64_t cap = plan->out_cap;
  if (int rc = ensure_out_staging(plan)) return rc;
  hipStream_t st = plan->stream;
  for (bool& u : plan->ev_used) u = false;
  if (plan->p.n_bits == 0) {
    if (int rc = fsk_empty_outputs(plan, B, plan->d_len, plan->d_sync)) return rc;
  } else {
    void* xs = nullptr;
    if (int rc = staging_buffer(plan, &xs)) return rc;
    if (x_stride == n)
      HIP_TRY(hipMemcpyAsync(xs, x, (size_t)(B * n * es), hipMemcpyHostToDevice, st));
    else
      HIP_TRY(hipMemcpy2DAsync(xs, (size_t)(n * es), x, (size_t)(x_stride * es), (size_t)(n * es), (size_t)B,
                               hipMemcpyHostToDevice, st));
    if (int rc = run_fsk(plan, xs, dtype, B, n, plan->d_out, cap, plan->d_len, plan->d_sync)) return rc;
  }
  if (out_stride == cap)
    HIP_TRY(hipMemcpyAsync(out, plan->d_out, (size_t)(B * cap), hipMemcpyDeviceToHost, st));
  else
    HIP_TRY(hipMemcpy2DAsync(out, (size_t)out_stride, plan->d_out, (size_t)cap, (size_t)std::min(out_stride, cap),
                             (size_t)B, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(out_len, plan->d_len, (size_t)B * 8, hipMemcpyDeviceToHost, st));
  HIP_TRY(hipMemcpyAsync(sync_idx, plan->d_sync, (size_t)B * 8, hipMemcpyDeviceToHost, st));
  return AMR_OK;
}

int amr_fsk_envelopes_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride,
                           double* mark_env, double* space_env) {
  if (!plan || (B && (!x || !mark_env || !space_env))) return fail(AMR_E_INVALID, "NULL argument");
  if (!dtype_size(dtype)) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (B == 0) return AMR_OK;
  const int64_t n = plan->p.n;
  std::vector<double> h((size_t)(B * n * 2));
  if (plan->p.lc.on) {
    // the envelopes at every sample need the natural layout's full passes: run
    // them on temporary buffers (a diagnostic entry, tests/test_gpu_fsk.py)
    const int64_t M = plan->fft.M;
    const int64_t ub = std::max(B * M * 16, fsk_bandpass_scratch_bytes(B, n, plan->p.pad));
    double2 *z = nullptr, *u = nullptr, *v = nullptr;
    void* xs = nullptr;
    hipError_t e = hipMalloc(&z, (size_t)(B * n * 16));
    if (e == hipSuccess) e = hipMalloc(&u, (size_t)ub);
    if (e == hipSuccess) e = hipMalloc(&v, (size_t)(B * M * 16));
    if (e == hipSuccess) e = hipMalloc(&xs, (size_t)(B * n * 8));
    int rc = e == hipSuccess ? copy_batch_h2d(xs, x, n * dtype_size(dtype), x_stride * dtype_size(dtype), B,
                                              plan->stream)
                             : fail(AMR_E_NOMEM, std::string("envelope buffers: ") + hipGetErrorString(e));
    if (rc == AMR_OK) {
      FskParams pn = plan->p;
      pn.lc = LiveCols{};
      std::swap(plan->z, z);
      std::swap(plan->u, u);
      std::swap(plan->v, v);
      std::swap(plan->p, pn);
      rc = run_fsk_front(plan, xs, dtype, B, n, true);
      if (rc == AMR_OK) {
        e = hipMemcpyAsync(h.data(), hilbert_out(plan->fft, plan->u, plan->v), h.size() * 8, hipMemcpyDeviceToHost,
                           plan->stream);
        if (e == hipSuccess) e = hipStreamSynchronize(plan->stream);
        if (e != hipSuccess) rc = fail(AMR_E_HIP, std::string("envelopes: ") + hipGetErrorString(e));
      }
      std::swap(plan->z, z);
      std::swap(plan->u, u);
      std::swap(plan->v, v);
      std::swap(plan->p, pn);
    }
    (void)hipStreamSynchronize(plan->stream);
    for (void* q : {(void*)z, (void*)u, (void*)v, xs})
      if (q) (void)hipFree(q);
    if (rc) return rc;
  } else {
    void* xs = nullptr;
    if (int rc = stage_input(plan, x, dtype, B, x_stride, &xs)) return rc;
    if (int rc = run_fsk_front(plan, xs, dtype, B, n, true)) return rc;
    HIP_TRY(hipMemcpyAsync(h.data(), hilbert_out(plan->fft, plan->u, plan->v), h.size() * 8, hipMemcpyDeviceToHost,
                           plan->stream));
    HIP_TRY(hipStreamSynchronize(plan->stream));
  }
  for (int64_t i = 0; i < B * n; ++i) {
    mark_env[i] = h[(size_t)(2 * i)];
    space_env[i] = h[(size_t)(2 * i + 1)];
  }
  return AMR_OK;
}

int amr_fft_c2c_host(const double* in, double* out, int64_t n, int64_t batch, int inverse, int device) {
  if (!in || !out || n < 1 || batch < 0) return fail(AMR_E_INVALID, "amr_fft_c2c_host: bad argument");
  if (batch == 0) return AMR_OK;
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  FftPlan f{};
  int rc = fft_plan_init(f, n, st, batch);
  double2 *x = nullptr, *u = nullptr, *v = nullptr;
  hipError_t e = hipSuccess;
  if (!rc) {
    e = hipMalloc(&x, (size_t)(batch * n * 16));
    if (e == hipSuccess) e = hipMalloc(&u, (size_t)(batch * f.M * 16));
    if (e == hipSuccess) e = hipMalloc(&v, (size_t)(batch * f.M * 16));
    if (e == hipSuccess) e = hipMemcpyAsync(x, in, (size_t)(batch * n * 16), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = fft_c2c(f, x, u, v, x, batch, inverse != 0, st);
    if (e == hipSuccess) e = hipMemcpyAsync(out, x, (size_t)(batch * n * 16), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  for (void* p : {(void*)x, (void*)u, (void*)v})
    if (p) (void)hipFree(p);
  fft_plan_free(f);
  (void)hipStreamDestroy(st);
  if (rc) return rc;
  HIP_TRY(e);
  return AMR_OK;
}

int amr_hilbert_host(const double* xr, double* analytic, int64_t n, int64_t batch, int device) {
  if (!xr || !analytic || n < 1 || batch < 0) return fail(AMR_E_INVALID, "amr_hilbert_host: bad argument");
  if (batch == 0) return AMR_OK;
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  FftPlan f{};
  int rc = fft_plan_init(f, n, st, batch);
  double2 *x = nullptr, *u = nullptr, *v = nullptr;
  hipError_t e = hipSuccess;
  std::vector<double> h((size_t)(batch * n * 2), 0.0);
  if (!rc) {
    for (int64_t i = 0; i < batch * n; ++i) h[(size_t)(2 * i)] = xr[i];
    e = hipMalloc(&x, (size_t)(batch * n * 16));
    if (e == hipSuccess) e = hipMalloc(&u, (size_t)(batch * f.M * 16));
    if (e == hipSuccess) e = hipMalloc(&v, (size_t)(batch * f.M * 16));
    if (e == hipSuccess) e = hipMemcpyAsync(x, h.data(), h.size() * 8, hipMemcpyHostToDevice, st);
    FftEpi store{};
    store.mode = kStore;
    if (e == hipSuccess) e = fft_hilbert(f, x, u, v, batch, store, st);
    if (e == hipSuccess)
      e = hipMemcpyAsync(h.data(), hilbert_out(f, u, v), h.size() * 8, hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
  }
  for (void* p : {(void*)x, (void*)u, (void*)v})
    if (p) (void)hipFree(p);
  fft_plan_free(f);
  (void)hipStreamDestroy(st);
  if (rc) return rc;
  HIP_TRY(e);
  for (int64_t i = 0; i < batch * n; ++i) {
    analytic[2 * i] = xr[i];
    analytic[2 * i + 1] = h[(size_t)(2 * i)];
  }
  return AMR_OK;
}

// pocketfft plans of one length on the device (plan struct + tables), for the
// one-shot host entries below
struct PfDev {
  PfLen L{};
  PfLen* dL = nullptr;
  double* pool = nullptr;
  ~PfDev() {
    if (dL) (void)hipFree(dL);
    if (pool) (void)hipFree(pool);
  }
};
int pf_dev_init(PfDev& D, int64_t n, double* tmp, hipStream_t st) {
  std::vector<double> pool;
  if (!pf_len_build(n, D.L, pool)) return fail(AMR_E_INVALID, "no pocketfft plan for length " + std::to_string(n));
  HIP_TRY(hipMalloc(&D.pool, pool.size() * 8 + 16));
  HIP_TRY(hipMalloc(&D.dL, sizeof(PfLen)));
  HIP_TRY(hipMemcpy(D.pool, pool.data(), pool.size() * 8, hipMemcpyHostToDevice));
  HIP_TRY(hipMemcpy(D.dL, &D.L, sizeof(PfLen), hipMemcpyHostToDevice));
  HIP_TRY(pf_finish(D.L, D.dL, D.pool, tmp, st));
  return AMR_OK;
}

int amr_resample_host(const double* x, int64_t nx, int64_t num, int64_t batch, double* y, int device) {
  if (!x || !y || nx < 1 || num < 1 || batch < 0) return fail(AMR_E_INVALID, "amr_resample_host: bad argument");
  if (batch == 0) return AMR_OK;
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  PfDev Dx, Dy;
  double *xd = nullptr, *yd = nullptr, *slots = nullptr;
  const int n_slots = (int)std::min<int64_t>(batch, 64);
  // scratch for the slots, and for pf_finish's transform before that
  const int64_t sd = std::max(pf_scratch_doubles_n(nx), pf_scratch_doubles_n(num)) + pf_even(std::max(nx, num));
  int rc = AMR_OK;
  hipError_t e = hipMalloc(&slots, (size_t)(n_slots * sd * 8));
  if (e == hipSuccess) e = hipMalloc(&xd, (size_t)(batch * nx * 8));
  if (e == hipSuccess) e = hipMalloc(&yd, (size_t)(batch * num * 8));
  if (e != hipSuccess) rc = fail(AMR_E_NOMEM, std::string("resample buffers: ") + hipGetErrorString(e));
  if (rc == AMR_OK) rc = pf_dev_init(Dx, nx, slots, st);
  if (rc == AMR_OK) rc = pf_dev_init(Dy, num, slots, st);
  if (rc == AMR_OK) {
    const int64_t slot = pf_resample_slot_doubles(Dx.L, Dy.L);
    e = hipMemcpyAsync(xd, x, (size_t)(batch * nx * 8), hipMemcpyHostToDevice, st);
    // irfft's 1/num (pocketfft: double(1 / long double num)), then numpy's y *= num / nx
    if (e == hipSuccess)
      e = launch_pf_resample(Dx.dL, Dx.pool, Dy.dL, Dy.pool, xd, nx, yd, num, batch, slots, slot, n_slots,
                             (double)(1.0L / (long double)num), (double)num / (double)nx, st);
    if (e == hipSuccess) e = hipMemcpyAsync(y, yd, (size_t)(batch * num * 8), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = fail(AMR_E_HIP, std::string("resample: ") + hipGetErrorString(e));
  }
  (void)hipStreamSynchronize(st);
  for (void* p : {(void*)xd, (void*)yd, (void*)slots})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(st);
  return rc;
}

int amr_hilbert_env_exact_host(const double* x, int64_t n, int64_t batch, double* env, int device) {
  if (!x || !env || n < 1 || batch < 0) return fail(AMR_E_INVALID, "amr_hilbert_env_exact_host: bad argument");
  if (batch == 0) return AMR_OK;
  HIP_TRY(hipSetDevice(device));
  hipStream_t st = nullptr;
  HIP_TRY(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
  PfDev D;
  double *xd = nullptr, *slots = nullptr;
  const int64_t sd = pf_even(n) + pf_scratch_doubles_n(n);   // the fused envelope keeps the spectrum in its slot
  // as the FSK exact path: up to 512 persistent workgroups within 2 GiB
  const int n_slots = (int)std::max<int64_t>(1, std::min<int64_t>({batch, 512, ((int64_t)1 << 31) / (sd * 8)}));
  int rc = AMR_OK;
  hipError_t e = hipMalloc(&slots, (size_t)(n_slots * sd * 8));
  if (e == hipSuccess) e = hipMalloc(&xd, (size_t)(batch * n * 8));
  if (e != hipSuccess) rc = fail(AMR_E_NOMEM, std::string("envelope buffers: ") + hipGetErrorString(e));
  if (rc == AMR_OK) rc = pf_dev_init(D, n, slots, st);
  if (rc == AMR_OK) {
    e = hipMemcpyAsync(xd, x, (size_t)(batch * n * 8), hipMemcpyHostToDevice, st);
    if (e == hipSuccess)
      e = launch_pf_hilbert_env(D.dL, D.pool, xd, n, batch, slots, sd, n_slots, (double)(1.0L / (long double)n),
                                pf_hilbert_lean(D.L), st);
    if (e == hipSuccess) e = hipMemcpyAsync(env, xd, (size_t)(batch * n * 8), hipMemcpyDeviceToHost, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    if (e != hipSuccess) rc = fail(AMR_E_HIP, std::string("exact envelopes: ") + hipGetErrorString(e));
  }
  (void)hipStreamSynchronize(st);
  for (void* p : {(void*)xd, (void*)slots})
    if (p) (void)hipFree(p);
  (void)hipStreamDestroy(st);
  return rc;
}

}  // extern "C"
