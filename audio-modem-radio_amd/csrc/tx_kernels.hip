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
//                   lane per stream, branch-free per symbol, payload bytes
//                   prefetched a batch ahead, phase[s][j] stored in 16-B pairs.
//   T2 k_tx_synth   4 consecutive samples per thread: sin(w[i] + phase) * env[i]
//                   rounded to float32 (and the WAV's int16), zero past the
//                   stream's natural length; 4 KiB per float4 store instruction.
// Every operation is the reference's IEEE double operation in its order
// (-ffp-contract=off): the tables and phases are bit-identical to numpy's.
// The one difference left is sin itself (ocml vs the host libm), a last-ulp
// matter in float64 that reaches the float32 output rarely (none of the
// reference fixtures' samples; tests/test_gpu_tx.py states the bound).
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

// (x + inc) % (2*pi) for the CPFSK recursion when x is known to lie in
// [0, 2^40): the exact fmod by one fused multiply-add with the right
// quotient (x - q*y is representable for the true q; a q off by one shows
// as r < 0 or r >= y and is corrected without a branch).
__device__ __forceinline__ double mod_two_pi_fast(double x, double y, double inv_y) {
  const double q = trunc(x * inv_y);
  const double r = fma(-q, y, x);
  const double qc = r < 0.0 ? q - 1.0 : (r >= y ? q + 1.0 : q);
  return fma(-qc, y, x);
}

// The symbols of one byte (MSB first), the reference's update per symbol, and
// their phases stored in 16-B pairs (GUARD: only those below n).
template <int MODE, bool FASTMOD, bool GUARD>
__device__ __forceinline__ void tx_byte(uint32_t byte, double& ph, double* __restrict__ out, int64_t& j, int64_t n,
                                        double inc0, double inc1) {
  constexpr int SPB = MODE == AMR_TX_QPSK ? 4 : 8;
  constexpr double kPi = 3.141592653589793;
  constexpr double kTwoPi = 2.0 * kPi;
  constexpr double kInvTwoPi = 1.0 / kTwoPi;
  double v[SPB];
#pragma unroll
  for (int k = 0; k < SPB; ++k) {
    if (MODE == AMR_TX_QPSK) {
      // phase_map (modem.py:160-165): 00 -> 0, 01 -> pi/2, 11 -> pi, 10 -> -pi/2,
      // i.e. m * (pi/2) with m = 0, 1, 2, -1: every product exact (power-of-2 scaling)
      const int hi = (byte >> (7 - 2 * k)) & 1, lo = (byte >> (6 - 2 * k)) & 1;
      const int m = lo ? hi + 1 : -hi;
      ph = ph + (double)m * (kPi / 2);               // current_phase += phase_change (+0.0 is exact)
      v[k] = ph;
    } else if (MODE == AMR_TX_BPSK) {
      ph = ph + (double)((byte >> (7 - k)) & 1) * kPi;   // current_phase += np.pi (or + 0.0)
      v[k] = ph;
    } else {
      v[k] = ph;                                     // the chunk uses the phase before the update
      const double x = ph + (((byte >> (7 - k)) & 1) ? inc0 : inc1);
      ph = FASTMOD ? mod_two_pi_fast(x, kTwoPi, kInvTwoPi) : py_mod(x, kTwoPi);
    }
  }
  if (!GUARD) {
#pragma unroll
    for (int k = 0; k < SPB; k += 2) *reinterpret_cast<double2*>(out + j + k) = make_double2(v[k], v[k + 1]);
  } else {
#pragma unroll
    for (int k = 0; k < SPB; ++k)
      if (j + k < n) out[j + k] = v[k];
  }
  j += SPB;
}

// T1: the phase recursion, lane per stream.  The symbols come from the
// preamble (as bytes: QPSK [0,0]*30+[1,1]*10 = 00 x7, 0F, FF, FF; BPSK [1,0]*40
// = AA x10; FSK AA x4) then the payload, read kTxBatch bytes at a time with the
// next batch in flight (one wave's loads touch 64 rows: the latency, not the
// bytes, is what the serial chain would otherwise wait on).  Full batches run
// without guards; the last bytes go one at a time.
constexpr int kTxBatch = 32;

template <int MODE, bool FASTMOD>
__global__ __launch_bounds__(64) void k_tx_phase(const uint8_t* __restrict__ data, int64_t stride,
                                                 const int64_t* __restrict__ n_bytes, int64_t n_streams, TxParams p,
                                                 double* __restrict__ phase) {
  constexpr int SPB = MODE == AMR_TX_QPSK ? 4 : 8;
  constexpr int PRE = MODE == AMR_TX_FSK ? 4 : 10;
  const int64_t s = (int64_t)blockIdx.x * kWave + threadIdx.x;
  if (s >= n_streams) return;
  int64_t nb = n_bytes[s];
  nb = nb < 0 ? 0 : (nb > stride ? stride : nb);
  const uint8_t* __restrict__ d = data + s * stride;
  const int64_t total = (int64_t)SPB * (PRE + nb);
  const int64_t n = total < p.sym_stride ? total : p.sym_stride;
  double* __restrict__ out = phase + s * p.sym_stride;
  double ph = 0.0;                                   // current_phase = 0
  int64_t j = 0;
#pragma unroll
  for (int q = 0; q < PRE; ++q) {
    const uint32_t byte = MODE == AMR_TX_QPSK ? (q < 7 ? 0x00u : q == 7 ? 0x0Fu : 0xFFu) : 0xAAu;
    tx_byte<MODE, FASTMOD, true>(byte, ph, out, j, n, p.inc0, p.inc1);
  }
  // payload bytes with a stored symbol (need), of which `full` store all SPB
  const int64_t left = n - j;
  int64_t need = left > 0 ? (left + SPB - 1) / SPB : 0;
  need = need < nb ? need : nb;
  int64_t full = left > 0 ? left / SPB : 0;
  full = full < need ? full : need;
  const int64_t nbat = full / kTxBatch;
  const int64_t last = nb > 0 ? nb - 1 : 0;          // loads clamp here instead of branching
  uint32_t nxt[kTxBatch];
  if (nbat > 0) {
#pragma unroll
    for (int t = 0; t < kTxBatch; ++t) nxt[t] = d[t];
  }
  for (int64_t b = 0; b < nbat; ++b) {
    const int64_t b0 = b * kTxBatch;
    uint32_t cur[kTxBatch];
#pragma unroll
    for (int t = 0; t < kTxBatch; ++t) cur[t] = nxt[t];
#pragma unroll
    for (int t = 0; t < kTxBatch; ++t) {
      const int64_t a = b0 + kTxBatch + t;
      nxt[t] = d[a < last ? a : last];
    }
#pragma unroll
    for (int t = 0; t < kTxBatch; ++t) tx_byte<MODE, FASTMOD, false>(cur[t], ph, out, j, n, p.inc0, p.inc1);
  }
  for (int64_t q = nbat * kTxBatch; q < need; ++q) tx_byte<MODE, FASTMOD, true>(d[q], ph, out, j, n, p.inc0, p.inc1);
}

// T2: 4 consecutive samples per thread (one 16-B store each; VEC: the rows
// allow it), the symbol index by one division per thread.  VALU-issue bound
// (~110 instructions per sample, half of them sin's FP64 work).
template <int MODE, bool VEC>
__global__ __launch_bounds__(256) void k_tx_synth(const uint8_t* __restrict__ data, int64_t stride,
                                                  const int64_t* __restrict__ n_bytes, TxParams p,
                                                  const double* __restrict__ phase, const double* __restrict__ tab,
                                                  float* __restrict__ out, int64_t out_stride,
                                                  int16_t* __restrict__ pcm, int64_t pcm_stride) {
  const int64_t s = blockIdx.y;
  int64_t nb = n_bytes[s];
  nb = nb < 0 ? 0 : (nb > stride ? stride : nb);
  const int64_t len = tx_symbols(MODE, nb) * p.sps;
  const uint8_t* __restrict__ d = data + s * stride;
  const double* __restrict__ ph = phase + s * p.sym_stride;
  const uint32_t sps = (uint32_t)p.sps;
  const int64_t k0 = (int64_t)blockIdx.x * 1024 + 4 * threadIdx.x;
  if (k0 >= p.n_out) return;
  uint32_t sym = (uint32_t)k0 / sps;
  uint32_t i = (uint32_t)k0 - sym * sps;
  float f[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) {
    f[u] = 0.0f;
    if (k0 + u < len) {
      if (MODE == AMR_TX_FSK) {
        const int bit = sym < 32 ? !(sym & 1) : (d[(sym - 32) >> 3] >> (7 - ((sym - 32) & 7))) & 1;
        const double w = bit ? tab[i] : tab[p.sps + i];
        f[u] = (float)sin(w + ph[sym]);            // np.array(out, dtype=np.float32)
        f[u] = f[u] * 0.9f;                        // ... * 0.9 (float32, NEP 50)
      } else {
        const double v = sin(tab[i] + ph[sym]) * tab[2 * p.sps + i];   // symbol * envelope
        f[u] = (float)v;
      }
    }
    if (++i == sps) {
      i = 0;
      ++sym;
    }
  }
  int16_t q[4];
#pragma unroll
  for (int u = 0; u < 4; ++u) q[u] = (int16_t)(int)(f[u] * 32767.0f);   // (arr * 32767).astype(np.int16)
  float* __restrict__ o = out + s * out_stride + k0;
  int16_t* __restrict__ c = pcm ? pcm + s * pcm_stride + k0 : nullptr;
  if (VEC && k0 + 4 <= p.n_out) {
    *reinterpret_cast<float4*>(o) = make_float4(f[0], f[1], f[2], f[3]);
    if (c) *reinterpret_cast<short4*>(c) = make_short4(q[0], q[1], q[2], q[3]);
  } else {
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (k0 + u < p.n_out) {
        o[u] = f[u];
        if (c) c[u] = q[u];
      }
    }
  }
}

template <int MODE>
static void launch_tx_mode(const TxParams& p, const uint8_t* data, int64_t stride, const int64_t* n_bytes,
                           int64_t n_streams, const double* tab, double* phase, float* out, int64_t out_stride,
                           int16_t* pcm, int64_t pcm_stride, hipStream_t st) {
  const dim3 pg((unsigned)((n_streams + kWave - 1) / kWave));
  // the branch-free fmod needs (phase + inc) in [0, 2^40): both increments in [0, 2^39)
  const bool fast = MODE != AMR_TX_FSK || (p.inc0 >= 0.0 && p.inc1 >= 0.0 && p.inc0 < 0x1p39 && p.inc1 < 0x1p39);
  if (fast)
    hipLaunchKernelGGL((k_tx_phase<MODE, true>), pg, dim3(kWave), 0, st, data, stride, n_bytes, n_streams, p, phase);
  else
    hipLaunchKernelGGL((k_tx_phase<MODE, false>), pg, dim3(kWave), 0, st, data, stride, n_bytes, n_streams, p, phase);
  const dim3 sg((unsigned)((p.n_out + 1023) / 1024), (unsigned)n_streams);
  const bool vec = (out_stride % 4) == 0 && ((uintptr_t)out % 16) == 0 &&
                   (!pcm || ((pcm_stride % 4) == 0 && ((uintptr_t)pcm % 8) == 0));
  if (vec)
    hipLaunchKernelGGL((k_tx_synth<MODE, true>), sg, dim3(256), 0, st, data, stride, n_bytes, p, phase, tab, out,
                       out_stride, pcm, pcm_stride);
  else
    hipLaunchKernelGGL((k_tx_synth<MODE, false>), sg, dim3(256), 0, st, data, stride, n_bytes, p, phase, tab, out,
                       out_stride, pcm, pcm_stride);
}

hipError_t launch_tx(const TxParams& p, const uint8_t* data, int64_t stride, const int64_t* n_bytes,
                     int64_t n_streams, double* work, float* out, int64_t out_stride, int16_t* pcm,
                     int64_t pcm_stride, hipStream_t st) {
  if (n_streams <= 0 || p.n_out <= 0) return hipSuccess;
  double* tab = work;
  double* phase = work + ((3 * p.sps + 1) & ~(int64_t)1);   // 16-B aligned rows (sym_stride is even)
  hipLaunchKernelGGL(k_tx_tables, dim3((unsigned)((p.sps + 255) / 256)), dim3(256), 0, st, p, tab);
  if (p.mode == AMR_TX_QPSK)
    launch_tx_mode<AMR_TX_QPSK>(p, data, stride, n_bytes, n_streams, tab, phase, out, out_stride, pcm, pcm_stride, st);
  else if (p.mode == AMR_TX_BPSK)
    launch_tx_mode<AMR_TX_BPSK>(p, data, stride, n_bytes, n_streams, tab, phase, out, out_stride, pcm, pcm_stride, st);
  else
    launch_tx_mode<AMR_TX_FSK>(p, data, stride, n_bytes, n_streams, tab, phase, out, out_stride, pcm, pcm_stride, st);
  return hipGetLastError();
}

}  // namespace amr
