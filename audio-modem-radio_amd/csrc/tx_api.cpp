// tx_api.cpp -- C ABI of the batched transmit side (include/amr.h).
//
// The host part of the reference's modulators: the scalar set-up each of
// them does before its per-symbol loop, restated with the same IEEE double
// operations (Python evaluates 2 * np.pi * f * t left to right):
//   sps  = int(samp_rate / baud)                  modem.py:35, 151
//   ramp = int(len(symbol) * 0.1)                 modem.py:58, 180
//   spb  = int(round(samp_rate * (1.0 / baud)))   modem.py:271-272 (round half even)
//   inc  = 2 * np.pi * f * (spb / samp_rate)      modem.py:292
// and the reference's error contract for them.  The sample work is
// tx_kernels.hip.
#include <hip/hip_runtime.h>

#include <cfenv>
#include <cmath>
#include <string>

#include "amr_internal.h"
#include "api_common.h"

namespace amr {
hipError_t launch_tx(const TxParams& p, const uint8_t* data, int64_t stride, const int64_t* n_bytes,
                     int64_t n_streams, double* work, float* out, int64_t out_stride, int16_t* pcm,
                     int64_t pcm_stride, hipStream_t st);
}  // namespace amr

using namespace amr;

namespace {

constexpr double kPi = 3.141592653589793;   // np.pi

int64_t tx_symbols(int mode, int64_t nb) {
  if (mode == AMR_TX_QPSK) return 40 + 4 * nb;
  if (mode == AMR_TX_BPSK) return 80 + 8 * nb;
  return 8 * (4 + nb);
}

// samples per symbol as the reference computes it; an AMR_E_* code (< 0 with
// the message set) when the reference raises for these parameters
int tx_setup(int mode, double baud, double f0, double f1, double fs, int64_t n_out, TxParams* p) {
  if (mode != AMR_TX_BPSK && mode != AMR_TX_QPSK && mode != AMR_TX_FSK)
    return fail(AMR_E_INVALID, "unknown modulation mode");
  if (baud == 0.0) return fail(AMR_E_INVALID, "float division by zero");
  if (!std::isfinite(baud) || !std::isfinite(fs)) return fail(AMR_E_INVALID, "baud and sample_rate must be finite");
  *p = TxParams{};
  p->mode = mode;
  p->fs = fs;
  p->n_out = n_out;
  if (mode == AMR_TX_FSK) {
    const double spb = std::nearbyint(fs * (1.0 / baud));   // int(round(samp_rate * bit_dur))
    p->sps = spb > 0 ? (int64_t)spb : 0;
    p->c0 = 2.0 * kPi * f0;
    p->c1 = 2.0 * kPi * f1;
    p->inc0 = 2.0 * kPi * f0 * ((double)(int64_t)spb / fs);
    p->inc1 = 2.0 * kPi * f1 * ((double)(int64_t)spb / fs);
  } else {
    const double q = fs / baud;
    const int64_t sps = (int64_t)q;                          // int(samp_rate / baud)
    p->sps = sps > 0 ? sps : 0;
    p->ramp = (int64_t)((double)p->sps * 0.1);               // int(len(symbol) * 0.1)
    p->c0 = 2.0 * kPi * f0;
    p->c1 = p->c0;
    if (p->sps > 0 && p->ramp == 0)                          // envelope[-0:] = linspace(1, 0, 0)
      return fail(AMR_E_INVALID, "could not broadcast input array from shape (0,) into shape (" +
                                     std::to_string(p->sps) + ",)");
  }
  p->sym_stride = p->sps > 0 ? (((n_out + p->sps - 1) / p->sps) + 1) & ~(int64_t)1 : 0;   // even: 16-B pairs
  return AMR_OK;
}

int64_t work_bytes(const TxParams& p, int64_t n) { return (3 * p.sps + n * p.sym_stride) * 8 + 256; }

}  // namespace

extern "C" {

int64_t amr_tx_samples(int mode, int64_t n_bytes, double baud, double sample_rate) {
  if (n_bytes < 0) return fail(AMR_E_INVALID, "n_bytes < 0");
  TxParams p;
  const int rc = tx_setup(mode, baud, 0.0, 0.0, sample_rate, 0, &p);
  if (rc) return rc;
  return tx_symbols(mode, n_bytes) * p.sps;
}

int64_t amr_tx_work_bytes(int mode, double baud, double sample_rate, int64_t n_streams, int64_t n_out) {
  if (n_streams < 0 || n_out < 0) return fail(AMR_E_INVALID, "negative size");
  TxParams p;
  const int rc = tx_setup(mode, baud, 0.0, 0.0, sample_rate, n_out, &p);
  if (rc) return rc;
  return work_bytes(p, n_streams);
}

int amr_modulate_device(amr_psk_plan* plan, int mode, double baud, double f0, double f1, double sample_rate,
                        const uint8_t* d_data, int64_t data_stride, const int64_t* d_n_bytes, int64_t n, float* d_out,
                        int64_t out_stride, int64_t n_out, int16_t* d_pcm, int64_t pcm_stride, void* d_work,
                        int64_t work_bytes_) {
  if (n < 0 || n_out < 0 || data_stride < 0 || out_stride < n_out || (d_pcm && pcm_stride < n_out))
    return fail(AMR_E_INVALID, "amr_modulate_device: bad argument");
  if (n && n_out && (!d_data || !d_n_bytes || !d_out))
    return fail(AMR_E_INVALID, "amr_modulate_device: NULL buffer");
  if (n > 65535) return fail(AMR_E_INVALID, "amr_modulate_device: at most 65535 streams per call");
  if (n_out > 0x7fffffffLL) return fail(AMR_E_INVALID, "amr_modulate_device: n_out >= 2^31");
  TxParams p;
  int rc = tx_setup(mode, baud, f0, f1, sample_rate, n_out, &p);
  if (rc) return rc;
  if (n == 0 || n_out == 0) return AMR_OK;
  if (p.sps > 0 && (!d_work || work_bytes_ < work_bytes(p, n)))
    return fail(AMR_E_INVALID, "amr_modulate_device: work buffer smaller than amr_tx_work_bytes()");
  int dev = 0;
  hipStream_t st = nullptr;
  rc = plan_stream(plan, &dev, &st);
  if (rc) return rc;
  if (p.sps == 0) {                                  // empty waveform: all padding
    HIP_TRY(hipMemset2DAsync(d_out, (size_t)out_stride * 4, 0, (size_t)n_out * 4, (size_t)n, st));
    if (d_pcm) HIP_TRY(hipMemset2DAsync(d_pcm, (size_t)pcm_stride * 2, 0, (size_t)n_out * 2, (size_t)n, st));
    return AMR_OK;
  }
  HIP_TRY(launch_tx(p, d_data, data_stride, d_n_bytes, n, (double*)d_work, d_out, out_stride, d_pcm, pcm_stride, st));
  return AMR_OK;
}

int amr_modulate_host(int mode, double baud, double f0, double f1, double sample_rate, const uint8_t* data,
                      int64_t data_stride, const int64_t* n_bytes, int64_t n, float* out, int64_t out_stride,
                      int64_t n_out, int16_t* pcm, int64_t pcm_stride) {
  if (n < 0 || n_out < 0 || data_stride < 0 || out_stride < n_out || (pcm && pcm_stride < n_out))
    return fail(AMR_E_INVALID, "amr_modulate_host: bad argument");
  if (n && (!n_bytes || (n_out && !out))) return fail(AMR_E_INVALID, "amr_modulate_host: NULL buffer");
  TxParams p;
  int rc = tx_setup(mode, baud, f0, f1, sample_rate, n_out, &p);
  if (rc) return rc;
  int64_t maxlen = 0;
  for (int64_t i = 0; i < n; ++i) {
    if (n_bytes[i] < 0 || n_bytes[i] > data_stride) return fail(AMR_E_INVALID, "n_bytes out of range");
    maxlen = n_bytes[i] > maxlen ? n_bytes[i] : maxlen;
  }
  if (maxlen > 0 && !data) return fail(AMR_E_INVALID, "amr_modulate_host: NULL data");
  if (n == 0 || n_out == 0) return AMR_OK;
  const int64_t stride = maxlen > 0 ? maxlen : 1;
  const int64_t wb = work_bytes(p, n);
  uint8_t* d_data = nullptr;
  int64_t* d_nb = nullptr;
  float* d_out = nullptr;
  int16_t* d_pcm = nullptr;
  void* d_work = nullptr;
  hipError_t e = hipMalloc(&d_data, (size_t)(n * stride));
  if (e == hipSuccess) e = hipMalloc(&d_nb, (size_t)n * 8);
  if (e == hipSuccess) e = hipMalloc(&d_out, (size_t)(n * n_out) * 4);
  if (e == hipSuccess && pcm) e = hipMalloc(&d_pcm, (size_t)(n * n_out) * 2);
  if (e == hipSuccess) e = hipMalloc(&d_work, (size_t)wb);
  if (e == hipSuccess && maxlen > 0)
    e = memcpy_rows(d_data, stride, data, data_stride, maxlen, n, hipMemcpyHostToDevice);
  if (e == hipSuccess) e = hipMemcpy(d_nb, n_bytes, (size_t)n * 8, hipMemcpyHostToDevice);
  if (e == hipSuccess) {
    rc = amr_modulate_device(nullptr, mode, baud, f0, f1, sample_rate, d_data, stride, d_nb, n, d_out, n_out, n_out,
                             d_pcm, n_out, d_work, wb);
    if (rc == AMR_OK) e = hipDeviceSynchronize();
  }
  if (e == hipSuccess && rc == AMR_OK)
    e = memcpy_rows(out, out_stride * 4, d_out, n_out * 4, n_out * 4, n, hipMemcpyDeviceToHost);
  if (e == hipSuccess && rc == AMR_OK && pcm)
    e = memcpy_rows(pcm, pcm_stride * 2, d_pcm, n_out * 2, n_out * 2, n, hipMemcpyDeviceToHost);
  for (void* q : {(void*)d_data, (void*)d_nb, (void*)d_out, (void*)d_pcm, d_work})
    if (q) (void)hipFree(q);
  if (rc) return rc;
  if (e != hipSuccess) return fail(AMR_E_HIP, std::string("amr_modulate_host: ") + hipGetErrorString(e));
  return AMR_OK;
}

}  // extern "C"
