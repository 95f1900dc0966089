// tx_kernels.hip -- batched transmit side for gfx950: the
// reference's modulators for many payloads at once, sample-for-sample.
//
//   bpsk_modulate   /root/reference/modem.py:28-65    DBPSK, +pi per 1-bit
//   qpsk_modulate   /root/reference/modem.py:138-186  DQPSK, Gray dibit steps
//   fsk_modulate    /root/reference/modem.py:270-295  CPFSK, phase mod 2*pi
//   wav_from_array  /root/reference/modem.py:360-368  int16(arr * 32767)
//
// Three launches per call:
//   T0 k_tx_tables  the per-symbol tables the reference rebuilds per symbol:
//                   w[i] = (2*pi*f) * (i / fs) and the 10 % linear ramps of
//                   np.linspace (numpy's own formula: i*step + start, the end
//                   point written as `stop`).  [3][sps] doubles.
//   T1 k_tx_phase   the phase recursion, which is a sequential float sum in the
//                   reference (current_phase += step, or CPFSK's
//                   phase = (phase + inc) % 2pi) and so stays sequential: one
//                   lane per stream, phase[s][j] per symbol into HBM.
//   T2 k_tx_synth   one thread per output sample: sin(w[i] + phase) * env[i],
//                   rounded to float32 (and the WAV's int16), zero past the
//                   stream's natural length.  1 KiB per store instruction.
// Every operation is the reference's IEEE double operation in its order
// (-ffp-contract=off): the tables and phases are bit-identical to numpy's.
// The one difference left is sin itself (ocml vs the host libm), a last-ulp
// matter in float64 that reaches the float32 output a few times per 1e8
// samples (tests/test_gpu_tx.py states the bound).
#include <math.h>

#include "amr_internal.h"
#include "amr.h"

namespace amr {

__device__ __forceinline__ int64_t tx_symbols(int mode, int64_t nb) {
  if (mode == AMR_TX_QPSK) return 40 + 4 * nb;   // ([0,0]*30 + [1,1]*10 + 8n bits) / 2
  if (mode == AMR_TX_BPSK) return 80 + 8 * nb;   // [1,0]*40 + 8n bits
  return 8 * (4 + nb);                           // b'\xAA'*4 + data, one chunk per bit
}

// T0: w0 = c0*t, w1 = c1*t, env (numpy.linspace, modem.py:56-61 / 180-183)
__global__ __launch_bounds__(256) void k_tx_tables(TxParams p, double* __restrict__ tab) {
  const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (i >= p.sps) return;
  const double t = (double)i / p.fs;               // np.arange(sps) / samp_rate
  tab[i] = p.c0 * t;                               // (2 * np.pi * f) * t
  tab[p.sps + i] = p.c1 * t;
  double e = 1.0;                                  // np.ones_like(symbol)
  const int64_t r = p.ramp;
  if (r > 0) {
    const double div = (double)(r - 1);
    if (i < r) {                                   // envelope[:ramp] = linspace(0, 1, ramp)
      e = (r > 1) ? (double)i * (1.0 / div) + 0.0 : (double)i * 1.0 + 0.0;
      if (r > 1 && i == r - 1) e = 1.0;
    }
    const int64_t j = i - (p.sps - r);
    if (j >= 0) {                                  // envelope[-ramp:] = linspace(1, 0, ramp)
      e = (r > 1) ? (double)j * (-1.0 / div) + 1.0 : (double)j * -1.0 + 1.0;
      if (r > 1 && j == r - 1) e = 0.0;
    }
  }
  tab[2 * p.sps + i] = e;
}

// phase % (2*pi) with Python / numpy float semantics (result has the sign of
// the divisor).  fmod is exact, so this is the reference's value.
__device__ __forceinline__ double py_mod(double x, double y) {
  double r = fmod(x, y);
  if (r != 0.0) {
    if ((r < 0.0) != (y < 0.0)) r += y;
  } else {
    r = copysign(0.0, y);
  }
  return r;
}

// T1: the phase recursion, lane per stream
__global__ __launch_bounds__(64) void k_tx_phase(const uint8_t* __restrict__ data, int64_t stride,
                                                 const int64_t* __restrict__ n_bytes, int64_t n_streams, TxParams p,
                                                 double* __restrict__ phase) {
  const int64_t s = (int64_t)blockIdx.x * kWave + threadIdx.x;
  if (s >= n_streams) return;
  int64_t nb = n_bytes[s];
  nb = nb < 0 ? 0 : (nb > stride ? stride : nb);
  const uint8_t* __restrict__ d = data + s * stride;
  const int64_t total = tx_symbols(p.mode, nb);
  const int64_t n = total < p.sym_stride ? total : p.sym_stride;
  double* __restrict__ out = phase + s * p.sym_stride;
  const double kPi = 3.141592653589793;
  double ph = 0.0;                                 // current_phase = 0
  if (p.mode == AMR_TX_QPSK) {
    // phase_map (modem.py:160-165): 00 -> 0, 01 -> pi/2, 11 -> pi, 10 -> -pi/2
    for (int64_t j = 0; j < n; ++j) {
      int dib;
      if (j < 30) dib = 0;
      else if (j < 40) dib = 3;
      else dib = (d[(j - 40) >> 2] >> (6 - 2 * ((j - 40) & 3))) & 3;
      const double step = dib == 0 ? 0.0 : dib == 1 ? kPi / 2 : dib == 2 ? -kPi / 2 : kPi;
      ph = ph + step;
      out[j] = ph;
    }
  } else if (p.mode == AMR_TX_BPSK) {
    for (int64_t j = 0; j < n; ++j) {
      const int bit = j < 80 ? !(j & 1) : (d[(j - 80) >> 3] >> (7 - ((j - 80) & 7))) & 1;
      if (bit) ph = ph + kPi;                      // current_phase += np.pi
      out[j] = ph;
    }
  } else {
    const double two_pi = 2.0 * kPi;
    for (int64_t j = 0; j < n; ++j) {
      const int bit = j < 32 ? !(j & 1) : (d[(j - 32) >> 3] >> (7 - ((j - 32) & 7))) & 1;
      out[j] = ph;                                 // the chunk uses the phase before the update
      ph = py_mod(ph + (bit ? p.inc0 : p.inc1), two_pi);
    }
  }
}

// T2: one thread per sample, 4 samples per thread at a 256 stride
__global__ __launch_bounds__(256) void k_tx_synth(const uint8_t* __restrict__ data, int64_t stride,
                                                  const int64_t* __restrict__ n_bytes, TxParams p,
                                                  const double* __restrict__ phase, const double* __restrict__ tab,
                                                  float* __restrict__ out, int64_t out_stride,
                                                  int16_t* __restrict__ pcm, int64_t pcm_stride) {
  const int64_t s = blockIdx.y;
  int64_t nb = n_bytes[s];
  nb = nb < 0 ? 0 : (nb > stride ? stride : nb);
  const int64_t len = tx_symbols(p.mode, nb) * p.sps;
  const uint8_t* __restrict__ d = data + s * stride;
  const double* __restrict__ ph = phase + s * p.sym_stride;
  const uint32_t sps = (uint32_t)p.sps;
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int64_t k = (int64_t)blockIdx.x * 1024 + r * 256 + threadIdx.x;
    if (k >= p.n_out) break;
    float f = 0.0f;
    if (k < len) {
      const uint32_t sym = (uint32_t)k / sps;
      const uint32_t i = (uint32_t)k - sym * sps;
      if (p.mode == AMR_TX_FSK) {
        const int bit = sym < 32 ? !(sym & 1) : (d[(sym - 32) >> 3] >> (7 - ((sym - 32) & 7))) & 1;
        const double w = bit ? tab[i] : tab[p.sps + i];
        f = (float)sin(w + ph[sym]);               // np.array(out, dtype=np.float32)
        f = f * 0.9f;                              // ... * 0.9 (float32, NEP 50)
      } else {
        const double v = sin(tab[i] + ph[sym]) * tab[2 * p.sps + i];   // symbol * envelope
        f = (float)v;
      }
    }
    out[s * out_stride + k] = f;
    if (pcm) pcm[s * pcm_stride + k] = (int16_t)(int)(f * 32767.0f);   // (arr * 32767).astype(np.int16)
  }
}

hipError_t launch_tx(const TxParams& p, const uint8_t* data, int64_t stride, const int64_t* n_bytes,
                     int64_t n_streams, double* work, float* out, int64_t out_stride, int16_t* pcm,
                     int64_t pcm_stride, hipStream_t st) {
  if (n_streams <= 0 || p.n_out <= 0) return hipSuccess;
  double* tab = work;
  double* phase = work + 3 * p.sps;
  hipLaunchKernelGGL(k_tx_tables, dim3((unsigned)((p.sps + 255) / 256)), dim3(256), 0, st, p, tab);
  hipLaunchKernelGGL(k_tx_phase, dim3((unsigned)((n_streams + kWave - 1) / kWave)), dim3(kWave), 0, st, data,
                     stride, n_bytes, n_streams, p, phase);
  hipLaunchKernelGGL(k_tx_synth, dim3((unsigned)((p.n_out + 1023) / 1024), (unsigned)n_streams), dim3(256), 0, st,
                     data, stride, n_bytes, p, phase, tab, out, out_stride, pcm, pcm_stride);
  return hipGetLastError();
}

}  // namespace amr
