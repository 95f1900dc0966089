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
#include <mutex>
#include <string>
#include <vector>

#include "amr_internal.h"
#include "api_common.h"
#include "fft.h"

namespace amr {
hipError_t launch_fsk_bandpass(int, const void*, int64_t, int64_t, double*, double2*, const FskParams&,
                               const FskIir&, hipStream_t);
hipError_t launch_fsk_decide(const uint8_t*, uint32_t*, int64_t, const FskParams&, hipStream_t);
int64_t fsk_bandpass_scratch_bytes(int64_t n_streams, int64_t n, int pad);
hipError_t launch_sync_pack(const uint32_t*, int64_t, int64_t, int64_t, uint8_t*, int64_t, int64_t*, int64_t*,
                            hipStream_t);
}  // namespace amr

using namespace amr;

namespace {

// Device FFT of one logical length n.
struct FftPlan {
  int64_t n = 0;
  int64_t M = 0;                 // transform length run: n, or the Bluestein length
  bool bluestein = false;
  FftDesc d{};                   // length M
  double2* tables = nullptr;     // [tw n2][tw n1][tw M][chirp n][bhat M]
  const double2* chirp = nullptr;
  const double2* bhat = nullptr;
};

void fft_plan_free(FftPlan& f) {
  if (f.tables) (void)hipFree(f.tables);
  f.tables = nullptr;
}

// Plans FFT_n; needs the plan's stream for the Bluestein kernel FFT.
int fft_plan_init(FftPlan& f, int64_t n, hipStream_t st) {
  static std::once_flag smem_once;
  static hipError_t smem_err = hipSuccess;
  std::call_once(smem_once, [] { smem_err = fft_configure_smem(); });
  HIP_TRY(smem_err);
  f.n = n;
  int n1 = 0, n2 = 0;
  if (fft_split(n, n1, n2)) {
    f.M = n;
  } else {
    f.bluestein = true;
    f.M = fft_good_size(2 * n - 1);
    if (f.M < 0 || !fft_split(f.M, n1, n2))
      return fail(AMR_E_INVALID, "FFT length " + std::to_string(n) + " exceeds the two-pass limit (Bluestein "
                                 "length <= " + std::to_string((int64_t)kFftMaxL * kFftMaxL) + ")");
  }
  const int64_t M = f.M;
  const int64_t nhi = (M + 255) / 256;
  // [tw n2][tw n1][W_M^t, t < 256][W_M^(256 t), t < nhi][chirp n][bhat M]
  const int64_t ntab = n2 + n1 + 256 + nhi + (f.bluestein ? n + M : 0);
  std::vector<double> host;
  host.reserve((size_t)(2 * ntab));
  auto put = [&](const std::vector<double>& w) { host.insert(host.end(), w.begin(), w.end()); };
  put(twiddles(n2, n2));
  put(twiddles(n1, n1));
  put(twiddles(M, 256));
  put(twiddles(M, nhi, 256));
  const int64_t off_chirp = n2 + n1 + 256 + nhi;
  std::vector<double> bw;
  if (f.bluestein) {
    // chirp w_j = exp(i pi j^2 / n); j^2 reduced mod 2n keeps the angle exact
    for (int64_t j = 0; j < n; ++j) {
      const int64_t r = (j * j) % (2 * n);
      const double a = M_PI * (double)r / (double)n;
      host.push_back(std::cos(a));
      host.push_back(std::sin(a));
    }
    // convolution kernel bw[m] = w_m, bw[M-m] = w_m (0 < m < n), zero elsewhere
    bw.assign((size_t)(2 * M), 0.0);
    const double* w = host.data() + 2 * off_chirp;
    for (int64_t m = 0; m < n; ++m) {
      bw[2 * m] = w[2 * m];
      bw[2 * m + 1] = w[2 * m + 1];
      if (m > 0) {
        bw[2 * (M - m)] = w[2 * m];
        bw[2 * (M - m) + 1] = w[2 * m + 1];
      }
    }
    host.resize((size_t)(2 * ntab), 0.0);
  }
  HIP_TRY(hipMalloc(&f.tables, (size_t)ntab * sizeof(double2)));
  HIP_TRY(hipMemcpy(f.tables, host.data(), (size_t)(2 * (off_chirp + (f.bluestein ? n : 0))) * 8,
                    hipMemcpyHostToDevice));
  const double2* t = f.tables;
  f.d.n = M;
  f.d.n1 = n1;
  f.d.n2 = n2;
  if (!fill_fft_len(f.d.a, n2, t) || !fill_fft_len(f.d.c, n1, t + n2))
    return fail(AMR_E_INVALID, "FFT factor plan failed for n=" + std::to_string(n));
  f.d.tw_lo = t + n2 + n1;
  f.d.tw_hi = t + n2 + n1 + 256;
  if (f.bluestein) {
    f.chirp = t + off_chirp;
    double2* bh = f.tables + off_chirp + n;
    f.bhat = bh;
    double2 *a = nullptr, *tmp = nullptr;
    HIP_TRY(hipMalloc(&a, (size_t)M * sizeof(double2)));
    hipError_t e = hipMalloc(&tmp, (size_t)M * sizeof(double2));
    if (e == hipSuccess) e = hipMemcpyAsync(a, bw.data(), (size_t)M * sizeof(double2), hipMemcpyHostToDevice, st);
    if (e == hipSuccess) e = launch_fft(a, tmp, bh, f.d, 1, false, st);
    if (e == hipSuccess) e = hipStreamSynchronize(st);
    (void)hipFree(a);
    if (tmp) (void)hipFree(tmp);
    HIP_TRY(e);
  }
  return AMR_OK;
}

// out = FFT_n(in) or IFFT_n(in).  u, v: [batch][M] scratch; in != u; out != v.
hipError_t fft_c2c(const FftPlan& f, const double2* in, double2* u, double2* v, double2* out, int64_t batch,
                   bool inverse, hipStream_t st) {
  if (!f.bluestein) return launch_fft(in, u, out, f.d, batch, inverse, st);
  FftEpi store{};
  store.mode = kStore;
  store.n = f.n;        // row stride of `out` (launch_fft_filter sets its own)
  hipError_t e = launch_bs_pre(in, u, f.chirp, f.n, f.M, batch, inverse, st);
  if (e == hipSuccess) e = launch_fft_filter(u, v, u, v, f.d, batch, kMulTab, f.bhat, store, st);
  if (e == hipSuccess) e = launch_bs_post(v, out, f.chirp, f.n, f.M, batch, inverse, store, st);
  return e;
}

// epi(IFFT_n(-i*sgn(k) * FFT_n(in))) = epi(H[in]), the Hilbert transform of
// each row (scipy.signal.hilbert(x).imag for real x).  u, v: [batch][M]
// scratch, in != u, v; a kStore / kEnvOut result lands in hilbert_out(f, u, v).
double2* hilbert_out(const FftPlan& f, double2* u, double2* v) { return f.bluestein ? v : u; }

hipError_t fft_hilbert(const FftPlan& f, const double2* in, double2* u, double2* v, int64_t batch, FftEpi epi,
                       hipStream_t st) {
  epi.n = f.n;
  if (!f.bluestein) return launch_fft_filter(in, u, v, u, f.d, batch, kHilbert, nullptr, epi, st);
  const int64_t n = f.n, M = f.M;
  FftEpi store{};
  store.mode = kStore;
  FftEpi hil{};
  hil.mode = kHilbert;
  hil.n = n;
  // forward: W = -i sgn(k) FFT_n(in) -> u (n-long rows)
  hipError_t e = launch_bs_pre(in, u, f.chirp, n, M, batch, false, st);
  if (e == hipSuccess) e = launch_fft_filter(u, v, u, v, f.d, batch, kMulTab, f.bhat, store, st);
  if (e == hipSuccess) e = launch_bs_post(v, u, f.chirp, n, M, batch, false, hil, st);
  // inverse: epi(IFFT_n(W)) -> v / cmp
  if (e == hipSuccess) e = launch_bs_pre(u, v, f.chirp, n, M, batch, true, st);
  if (e == hipSuccess) e = launch_fft_filter(v, u, v, u, f.d, batch, kMulTab, f.bhat, store, st);
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
  double2* z = nullptr;        // [B][n]
  double2* u = nullptr;        // [B][M]  (also F1's checkpoint scratch)
  double2* v = nullptr;        // [B][M]
  uint8_t* cmp = nullptr;      // [B][bits_stride] packed compare bits (fft.h fft_bits_stride)
  uint32_t* words = nullptr;   // [B][n_words]
  int64_t scratch_bytes = 0;
  // staging for the host API
  void* d_x = nullptr;
  uint8_t* d_out = nullptr;
  int64_t* d_len = nullptr;
  int64_t* d_sync = nullptr;
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
  for (void* p : {(void*)pl->z, (void*)pl->u, (void*)pl->v, (void*)pl->cmp, (void*)pl->words, pl->d_x,
                  (void*)pl->d_out, (void*)pl->d_len, (void*)pl->d_sync})
    if (p) (void)hipFree(p);
  fft_plan_free(pl->fft);
  for (auto& e : pl->ev)
    for (auto& h : e)
      if (h) (void)hipEventDestroy(h);
  if (pl->stream) (void)hipStreamDestroy(pl->stream);
  delete pl;
}

// F1, F2: x -> cmp (or -> the two envelopes in hilbert_out(u, v) when env_out).  Caller holds mu.
int run_fsk_front(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, bool env_out) {
  hipStream_t st = pl->stream;
  auto mark = [&](int slot, int which) -> hipError_t {
    if (!pl->timing) return hipSuccess;
    pl->ev_used[slot] = true;
    return hipEventRecord(pl->ev[slot][which], st);
  };
  HIP_TRY(mark(AMR_TF_BANDPASS, 0));
  HIP_TRY(launch_fsk_bandpass(dtype, d_x, x_stride, B, reinterpret_cast<double*>(pl->u), pl->z, pl->p, pl->f, st));
  HIP_TRY(mark(AMR_TF_BANDPASS, 1));
  FftEpi env{};
  env.mode = env_out ? kEnvOut : kEnvelope;
  env.z = pl->z;
  env.bits = pl->cmp;
  env.bits_stride = pl->p.bits_stride;
  // one timing slot for the whole Hilbert filter (column, middle and final row passes)
  HIP_TRY(mark(AMR_TF_HILBERT, 0));
  HIP_TRY(fft_hilbert(pl->fft, pl->z, pl->u, pl->v, B, env, st));
  HIP_TRY(mark(AMR_TF_HILBERT, 1));
  return AMR_OK;
}

int run_fsk(amr_fsk_plan* pl, const void* d_x, int dtype, int64_t B, int64_t x_stride, uint8_t* d_out,
            int64_t out_stride, int64_t* d_len, int64_t* d_sync) {
  if (B < 0 || B > pl->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (dtype_size(dtype) == 0) return fail(AMR_E_INVALID, "unknown dtype");
  if (x_stride < pl->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (out_stride < pl->out_cap - 1 || out_stride < 1) return fail(AMR_E_INVALID, "out_stride too small");
  for (bool& u : pl->ev_used) u = false;
  if (B == 0) return AMR_OK;
  hipStream_t st = pl->stream;
  if (pl->p.n_bits == 0) {
    // no decision window (sps // 4 == 0): empty bit string -> b''   (modem.py:320-323)
    HIP_TRY(hipMemsetAsync(d_len, 0, (size_t)B * 8, st));
    HIP_TRY(hipMemsetAsync(d_sync, 0xFF, (size_t)B * 8, st));
    return AMR_OK;
  }
  if (int rc = run_fsk_front(pl, d_x, dtype, B, x_stride, false)) return rc;
  if (pl->timing) {
    pl->ev_used[AMR_TF_DECIDE] = true;
    HIP_TRY(hipEventRecord(pl->ev[AMR_TF_DECIDE][0], st));
  }
  HIP_TRY(launch_fsk_decide(pl->cmp, pl->words, B, pl->p, st));
  HIP_TRY(launch_sync_pack(pl->words, pl->p.n_words, pl->p.n_bits, B, d_out, out_stride, d_len, d_sync, st));
  if (pl->timing) HIP_TRY(hipEventRecord(pl->ev[AMR_TF_DECIDE][1], st));
  return AMR_OK;
}

int stage_input(amr_fsk_plan* pl, const void* x, int dtype, int64_t B, int64_t x_stride) {
  const int64_t es = dtype_size(dtype);
  const int64_t n = pl->p.n;
  if (!pl->d_x) HIP_TRY(hipMalloc(&pl->d_x, (size_t)(pl->max_streams * n * 8)));
  HIP_TRY(hipMemcpy2DAsync(pl->d_x, (size_t)(n * es), x, (size_t)(x_stride * es), (size_t)(n * es), (size_t)B,
                           hipMemcpyHostToDevice, pl->stream));
  return AMR_OK;
}

}  // namespace

extern "C" {

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
  FskParams& p = pl->p;
  p.n = n;
  p.sps = sps;
  p.nt = nt;
  p.pad = 3 * nt;
  const int64_t q = sps / 4, half = sps / 2;
  p.n_bits = (q > 0 && n > half) ? (n - half + sps - 1) / sps : 0;
  p.n_words = p.n_bits > 0 ? (p.n_bits + 31) / 32 : 1;
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
  pl->out_cap = p.n_bits / 8 + 1;
  e = hipStreamCreateWithFlags(&pl->stream, hipStreamNonBlocking);
  if (e != hipSuccess) {
    fsk_plan_free(pl);
    return fail(AMR_E_HIP, std::string("hipStreamCreate: ") + hipGetErrorString(e));
  }
  if (int rc = fft_plan_init(pl->fft, n, pl->stream)) {
    fsk_plan_free(pl);
    return rc;
  }
  const int64_t M = pl->fft.M;
  p.rn1 = pl->fft.bluestein ? n : pl->fft.d.n1;
  p.rn2 = pl->fft.bluestein ? 1 : pl->fft.d.n2;
  p.bits_stride = fft_bits_stride(p.rn1, p.rn2);
  p.inv_rn1 = 1.0f / (float)p.rn1;
  const int64_t s1_bytes = fsk_bandpass_scratch_bytes(max_streams, n, p.pad);
  struct A { void** ptr; int64_t bytes; };
  const A allocs[] = {
      {(void**)&pl->z, max_streams * n * 16},
      {(void**)&pl->u, std::max(max_streams * M * 16, s1_bytes)},
      {(void**)&pl->v, max_streams * M * 16},
      {(void**)&pl->cmp, max_streams * p.bits_stride},
      {(void**)&pl->words, max_streams * p.n_words * 4},
  };
  for (const A& a : allocs) {
    e = hipMalloc(a.ptr, (size_t)a.bytes);
    if (e != hipSuccess) {
      fsk_plan_free(pl);
      return fail(AMR_E_NOMEM, "hipMalloc(" + std::to_string(a.bytes) + " B): " + hipGetErrorString(e));
    }
    pl->scratch_bytes += a.bytes;
  }
  *out = pl;
  return AMR_OK;
}

int amr_fsk_plan_destroy(amr_fsk_plan* plan) {
  fsk_plan_free(plan);
  return AMR_OK;
}
int64_t amr_fsk_plan_out_capacity(const amr_fsk_plan* plan) { return plan ? plan->out_cap : -1; }
int64_t amr_fsk_plan_scratch_bytes(const amr_fsk_plan* plan) { return plan ? plan->scratch_bytes : -1; }
int64_t amr_fsk_plan_fft_length(const amr_fsk_plan* plan) { return plan ? plan->fft.M : -1; }

int amr_fsk_plan_synchronize(amr_fsk_plan* plan) {
  if (!plan) return fail(AMR_E_INVALID, "plan is NULL");
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
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

int amr_fsk_plan_timings(amr_fsk_plan* plan, float* ms, int count) {
  if (!plan || !ms) return fail(AMR_E_INVALID, "NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  HIP_TRY(hipStreamSynchronize(plan->stream));
  for (int i = 0; i < count && i < AMR_TF_COUNT; ++i) {
    ms[i] = -1.0f;
    if (plan->timing && plan->ev_used[i]) HIP_TRY(hipEventElapsedTime(&ms[i], plan->ev[i][0], plan->ev[i][1]));
  }
  return AMR_OK;
}

int amr_fsk_demod_device(amr_fsk_plan* plan, const void* d_x, int dtype, int64_t n_streams, int64_t x_stride,
                         uint8_t* d_out, int64_t out_stride, int64_t* d_out_len, int64_t* d_sync_idx) {
  if (!plan || (n_streams && (!d_x || !d_out || !d_out_len || !d_sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_device: NULL argument");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  return run_fsk(plan, d_x, dtype, n_streams, x_stride, d_out, out_stride, d_out_len, d_sync_idx);
}

int amr_fsk_demod_host(amr_fsk_plan* plan, const void* x, int dtype, int64_t B, int64_t x_stride, uint8_t* out,
                       int64_t out_stride, int64_t* out_len, int64_t* sync_idx) {
  if (!plan || (B && (!x || !out || !out_len || !sync_idx)))
    return fail(AMR_E_INVALID, "amr_fsk_demod_host: NULL argument");
  if (!dtype_size(dtype)) return fail(AMR_E_INVALID, "unknown dtype");
  std::lock_guard<std::mutex> lk(plan->mu);
  HIP_TRY(hipSetDevice(plan->device));
  if (B > plan->max_streams) return fail(AMR_E_CAPACITY, "batch exceeds plan max_streams");
  if (x_stride < plan->p.n) return fail(AMR_E_INVALID, "x_stride < n_samples");
  if (B == 0) return AMR_OK;
  const int64_t cap = plan->out_cap;
  if (int rc = stage_input(plan, x, dtype, B, x_stride)) return rc;
  if (!plan->d_out) {
    HIP_TRY(hipMalloc(&plan->d_out, (size_t)(plan->max_streams * cap)));
    HIP_TRY(hipMalloc(&plan->d_len, (size_t)plan->max_streams * 8));
    HIP_TRY(hipMalloc(&plan->d_sync, (size_t)plan->max_streams * 8));
  }
  if (int rc = run_fsk(plan, plan->d_x, dtype, B, plan->p.n, plan->d_out, cap, plan->d_len, plan->d_sync)) return rc;
  HIP_TRY(hipMemcpy2DAsync(out, (size_t)out_stride, plan->d_out, (size_t)cap,
                           (size_t)(out_stride < cap ? out_stride : cap), (size_t)B, hipMemcpyDeviceToHost,
                           plan->stream));
  HIP_TRY(hipMemcpyAsync(out_len, plan->d_len, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipMemcpyAsync(sync_idx, plan->d_sync, (size_t)B * 8, hipMemcpyDeviceToHost, plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
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
  if (int rc = stage_input(plan, x, dtype, B, x_stride)) return rc;
  if (int rc = run_fsk_front(plan, plan->d_x, dtype, B, n, true)) return rc;
  std::vector<double> h((size_t)(B * n * 2));
  HIP_TRY(hipMemcpyAsync(h.data(), hilbert_out(plan->fft, plan->u, plan->v), h.size() * 8, hipMemcpyDeviceToHost,
                         plan->stream));
  HIP_TRY(hipStreamSynchronize(plan->stream));
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
  int rc = fft_plan_init(f, n, st);
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
  int rc = fft_plan_init(f, n, st);
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

}  // extern "C"
