// amr_internal.h -- shared between the HIP kernels and the C-ABI runtime.
//
// Work decomposition:
//   * a "group" is 64 consecutive streams; one wave64 owns a group in the
//     band-pass kernel (lane = stream) and two waves own it in the low-pass
//     kernels (lane = stream x {re, im}).
//   * every intermediate lives in HBM TIME-MAJOR inside its group, so the 64
//     lanes of a wave touch one contiguous 512 B / 1 KiB row per sample step.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace amr {

constexpr int kWave = 64;
constexpr int kMaxTaps = 16;

enum DType : int { kF32 = 0, kF64 = 1, kI16 = 2 };
enum PskKind : int { kQpsk = 0, kBpsk = 1 };

// One IIR section as scipy.signal.lfilter sees it (a[0] == 1).
struct Iir {
  int nt;                 // taps (order + 1)
  double b[kMaxTaps];
  double a[kMaxTaps];
  double zi[kMaxTaps];    // scipy.signal.lfilter_zi(b, a)
};

// Everything a PSK launch needs besides the buffers.  Passed by value as a
// kernel argument, so the coefficients arrive in SGPRs.
struct PskParams {
  int64_t n;              // samples per stream
  int64_t m1;             // n + 2*pad1 (band-pass extended length)
  int64_t m2;             // n + 2*pad2 (low-pass extended length)
  int64_t sps;            // samples per symbol
  int64_t first;          // index of the first symbol sample
  int64_t n_sym;          // S = len(baseband[first::sps])
  int64_t n_bits;         // L = (S-1) * bits_per_symbol   (0 when S < 2)
  int64_t n_words;        // 32-bit words per stream in the bit buffer
  int pad1, pad2;
  int kind;               // PskKind
  int bp_zero_odd;        // 1: b[1], b[3], ... are all +0.0 (band-pass symmetry)
  int bp_sym;             // 1: 9 taps with b[8] == b[0] and b[6] == b[2] bit for bit
  int lp_sym;             // 1: 5 taps with b[4] == b[0] and b[3] == b[1] bit for bit
  // the lane layout's float32 hand-off (PskBuffers::f32f):
  // |symbol error| <= f32_margin * (the stream's max |f|) + 2^-120 when the
  // low-pass reads f rounded to float32 (api.cpp f32_design; 0: not allowed)
  double f32_margin;
};

// Pointers of one batch launch (device memory).
struct PskBuffers {
  const void* x;          // [B][x_stride] input samples
  int64_t x_stride;       // elements
  int dtype;
  int64_t n_streams;      // B
  int inflight;           // batches the caller keeps in flight (amr_psk_plan_set_inflight), >= 1
  const double* lo;       // [n][4]: (lo_re, -(0*lo_im), lo_im, 0*lo_re)
  const double* lo2;      // [2][n]: lo_re[n], lo_im[n] (the multipliers alone)
  double* s1;             // band-pass forward output  [G][m1p/2][64][2]
  double* s2;             // band-pass output f        [G][2][n2][32][2]
  double* s3;             // low-pass forward output   [2G][m2p/2][64][2]
  uint32_t* words;        // [B][n_words] bit buffer, MSB first
  int32_t* flags;         // [B] 1 => take the exact complex low-pass path
  int32_t* bp_flags;      // [B] 1 => the band-pass skipped its zero taps where that is not exact (lane kernels)
  uint8_t* out;           // [B][out_stride] packed bytes
  int64_t out_stride;
  int64_t* out_len;       // [B]
  int64_t* sync_idx;      // [B]
  const int32_t* gate;    // non-null: every kernel of the launch exits at once while *gate == 0
                          // (the time-split layout's serial fallback, api.cpp run_psk)
  // lane layout, float32 hand-off: the band-pass stores f rounded to float32
  // (half of each group's s2 slot) and its per-stream max |f| in fpeak; the
  // fused low-pass slicer flags (flags and bp_flags) every stream with a
  // decision inside the rounding's margin, whose group the band-pass fix-up
  // then recomputes in float64 for K3x / K4a
  int f32f;
  double* fpeak;          // [B]
  // the band-pass input's odd extension as the caller's dtype formed it
  // (odd_ext.h): [B][2 * pad1] (the left pad, then the right), or null
  const double* edge;
};

// the time-split strict bound's block of outputs (split_strict.h, psk_split_kernels.hip KB)
constexpr int kStrictBlk = 16;

// PSK time-split layout (psk_split_kernels.hip): each filtfilt
// pass cut into chunks of L outputs, one lane per chunk, each started w
// samples early from a zero state; decisions kept where the symbols' error
// bound kappa * peak|x| cannot move them, the rest flagged for the serial path.
struct PskSplit {
  int64_t L;              // outputs per chunk, every pass
  int64_t w1, w2;         // warm-up samples: band-pass, low-pass passes
  int64_t c1, c2;         // chunks per stream: ceil(m1 / L), ceil(m2 / L)
  double kappa;           // |symbol error| <= kappa * peak|ext x| (api.cpp split_design)
  double* y1;             // [B][m1] band-pass forward output (the plan's s1)
  double* f;              // [B][n] band-pass output (s2)
  double* y3;             // [B][2][m2] low-pass forward outputs, re then im (s3)
  double* sym;            // [B][S][re, im] symbol samples (s1, after the band-pass)
  unsigned long long* peak;   // [B] bits of max |ext x| (cleared per launch)
  int32_t* flag;          // [B] 1: a decision inside the margin (cleared per launch)
  int32_t* count;         // [1] flagged streams: the serial fallback's gate
  // band-pass chunk start states by convolution (KS0) instead
  // of w1-step warm-ups: conv = 1 uses them
  int conv;
  const double* ktab;     // [w1][8] state weights of past inputs (iir_design.h split_state_tables)
  const double* z0tab;    // [w1 + 1][8] scipy's zi state after t zero inputs
  double* zs;             // [B][c1][8] start states, KS0 -> KS1 (then reused for KS2)
  // STRICT mode (split_strict.h): the decisions' margin from a
  // bound that holds for every input instead of kappa * peak.  KS0 adds each
  // chunk start's error bound, KS1 / KS2 each step's rounding bound
  //   D = u2 sum_{i>=1} |z_i| + kx |x| + ky |y|
  // and their maxima per stream to bnd; KS5 turns them into a bound per symbol
  int strict;
  unsigned long long* bnd;   // [B][8] bits (cleared per launch): D1max, -, max|y1|, D2max, -, max|f|
  const double* kabs;        // [w1] sum_i |K_i[m]|
  const double* z0abs;       // [w1 + 1] sum_i |Z0_i[t]|
  const double* lpc;         // [n_sym] the band-pass error's reach to symbol k (the low-pass stage)
  double gam;                // KS0's dot-product rounding factor (gamma_n + the tables' 2u)
  double u2, kx, ky;         // the step bound's constants
  double g1x, gmax;          // 1 + sum_m max_j |g_j(m)|, its max
  double hz, tk, zi_sum, zb; // ||h||_1 + max|tz|; truncation per unit peak; sum|zi|; state sum per unit peak
  double c3;                 // the low-pass's own rounding, truncation, extension rounding per unit P3
  // the block bound (KB; split_strict.h kStrictBlk): kernels and their cut remainders
  const double *kW, *kK12, *kHS, *kGS, *kTZ;
  int nw, nk, k12_off, nh, nz;
  double w_tail, k12_tail, hs_tail, tz_tail, lp_tail;
  int64_t lp_rad;
  // per-stream scratch (stride sstride doubles): D1 blocks [nb1] | D2 blocks [nb1] | chunk start bounds
  // pass 1 [c1] | pass 2 [c1] | E1 blocks [nb1] | S1 blocks [nb1] | E2 blocks [nb1] | X blocks [nbs] |
  // e(k) [n_sym] | scalars [4]: E1max, Fmax, Xmax, P3 (negative: the caps failed, the stream is flagged)
  double* sc;
  int64_t sstride, nb1, nbs;
  double* ebound;            // diagnostic (amr_psk_split_bounds_host): copy e(k) and the scalars out
};

// offsets into PskSplit::sc
__host__ __device__ inline int64_t strict_off_d1(const PskSplit&) { return 0; }
__host__ __device__ inline int64_t strict_off_d2(const PskSplit& s) { return s.nb1; }
__host__ __device__ inline int64_t strict_off_ds1(const PskSplit& s) { return 2 * s.nb1; }
__host__ __device__ inline int64_t strict_off_ds2(const PskSplit& s) { return 2 * s.nb1 + s.c1; }
__host__ __device__ inline int64_t strict_off_e1(const PskSplit& s) { return 2 * s.nb1 + 2 * s.c1; }
__host__ __device__ inline int64_t strict_off_s1(const PskSplit& s) { return 3 * s.nb1 + 2 * s.c1; }
__host__ __device__ inline int64_t strict_off_e2(const PskSplit& s) { return 4 * s.nb1 + 2 * s.c1; }
__host__ __device__ inline int64_t strict_off_x(const PskSplit& s) { return 5 * s.nb1 + 2 * s.c1; }
__host__ __device__ inline int64_t strict_off_e(const PskSplit& s) { return 5 * s.nb1 + 2 * s.c1 + s.nbs; }

// FSK live-column layout.  A four-step length n = n1 * n2
// (sample i = j1 + n1 * j2) with n1 % sps == 0: every decision window of
// fsk_demodulate (bits[i - sps//4 : i + sps//4] at i = sps//2 + k*sps,
// modem.py:320-321) holds samples whose residue mod sps lies in
// [w0, w0 + nw), w0 = sps//2 - sps//4, nw = 2*(sps//4) -- whole columns j1
// of the four-step grid ("live" columns; 120 of 300 at sps 10).  The other
// columns feed no decision.  Per stream the filter output z is stored as
//   L: [j2][l]  the live columns  (nl = n1 / sps * nw of them)
//   D: [j2][d]  the dead columns  (nd = n1 - nl), right after L
// and the Hilbert filter's intermediates are kept only where a later pass
// reads them (fsk_api.cpp, fft_kernels.hip *_live kernels).
struct LiveCols {
  int on;                 // 0: natural layout [i]
  int n1, n2;
  int sps, w0, nw;        // live residues w0 .. w0 + nw - 1 (mod sps)
  int nl, nd;             // live / dead column counts
  float inv_n1, inv_sps, inv_nw, inv_ndp;   // reciprocals for lc_div (ndp = sps - nw)
  int prune;              // the middle pass computes only the live outputs of its last stage
};

// floor(i / d) for 0 <= i < 2^20 given inv = 1/d rounded to float, d <= 625:
// (i + 0.5) / d is >= 0.5/d away from an integer, the float product errs by
// < 2^-22 * i / d <= 0.25 / d (plan creation checks every index it uses)
__host__ __device__ inline int lc_div(int i, float inv) { return (int)(((float)i + 0.5f) * inv); }

// column j1 -> its index among the live (l) or dead (d) columns
__host__ __device__ inline int lc_col_pos(const LiveCols& m, int j1, bool& live) {
  const int a = lc_div(j1, m.inv_sps);
  const int v = j1 - a * m.sps;
  live = (unsigned)(v - m.w0) < (unsigned)m.nw;
  return live ? a * m.nw + (v - m.w0) : a * (m.sps - m.nw) + (v < m.w0 ? v : v - m.nw);
}
__host__ __device__ inline int lc_live_col(const LiveCols& m, int l) {
  const int a = lc_div(l, m.inv_nw);
  return a * m.sps + m.w0 + (l - a * m.nw);
}
__host__ __device__ inline int lc_dead_col(const LiveCols& m, int d) {
  const int ndp = m.sps - m.nw;
  const int a = lc_div(d, m.inv_ndp);
  const int v = d - a * ndp;
  return a * m.sps + (v < m.w0 ? v : v + m.nw);
}
// sample i of a stream -> its offset in the stream's [L | D] block
__host__ __device__ inline int64_t lc_zoff(const LiveCols& m, int i) {
  const int j2 = lc_div(i, m.inv_n1);
  bool live;
  const int pos = lc_col_pos(m, i - j2 * m.n1, live);
  return live ? (int64_t)j2 * m.nl + pos : (int64_t)m.nl * m.n2 + (int64_t)j2 * m.nd + pos;
}

// FSK (fsk_kernels.hip): both tones' band-pass filters, lane = (stream, tone)
struct FskParams {
  int64_t n;        // samples per stream
  int64_t sps;      // int(fs / baud)
  int64_t n_bits;   // decided bits per stream
  int64_t n_words;
  int nt;           // band-pass taps (7)
  int pad;          // 3 * nt
  int64_t rn1, rn2; // compare-bit layout (fft.h fft_bits_stride)
  int64_t bits_stride;
  float inv_rn1;
  LiveCols lc;      // lc.on: z and the compare bits in the live-column layout
  double* amb;       // non-null: F1 writes [B] each stream's ambiguity scale (amb_scale) and
                    // clears xflags; F2's last pass sets bit s of xflags[s / 32] for a stream
                    // with a compare inside the margin, F3 then reads its bits from xbits
                    // (the exact path, fsk_exact_kernels.hip)
  uint32_t* xflags;
  const uint8_t* xbits;
  int force_exact;  // exact mode 2 (amr_fsk_plan_set_exact_mode): every stream's scale +inf, all go exact
  const int32_t* xlist;   // F1 list mode (the exact path): z row r <- x row xlist[r], r < *xcount
  const int32_t* xcount;
  const double* edge;     // the odd extension as the caller's dtype formed it (odd_ext.h): [B][2 * pad] or null
  double tau;             // F2's margin scale (fsk_api.cpp fsk_fft_bound: >= kAmbTau, a standard FFT bound)
};

// F2's ambiguity margin: |env_mark - env_space| <= 2 tau peak|x| is within
// reach of the fast path's and pocketfft's rounding.
// F1 computes scipy's filtfilt bit for bit, so the envelopes differ from the
// reference's by the two FFTs' rounding alone: measured <= 4.3e-15 peak|x|
// (two-pass and Bluestein lengths, 300-9600 Bd).  A plan's tau (FskParams::tau)
// is the larger of kAmbTau = 2^-36 (>= 3000 times the measured difference)
// and a standard FFT rounding bound for its length and filters (fsk_api.cpp
// fsk_fft_bound, round 6: ~13 x 2^-36 at n = 96000)
constexpr double kAmbTau = 0x1p-36;
// c = 8 (tau peak)^2 (fft_kernels.hip env_ambiguous compares squares);
// -1 for a stream of exact zeros (both paths' envelopes are exact zeros),
// +inf for tiny / huge / non-finite input (every compare goes exact)
__host__ __device__ inline double amb_scale(double peak, double tau = kAmbTau) {
  if (peak == 0.0) return -1.0;
  if (!(peak >= 0x1p-400 && peak <= 0x1p400)) return __builtin_inf();
  const double d = tau * peak;
  return 8.0 * d * d;
}

// One filter's strict band-pass design as the kernels read it (split_strict.h
// strict_design_bp; the FSK split's strict mode holds one per tone): the
// convolution-start bound tables, the block kernels and their cut remainders,
// and the per-step / per-pass constants
struct StrictBp {
  const double* kabs;         // [w]
  const double* z0abs;        // [w + 1]
  const double *W, *K12, *HS, *GS, *TZ;
  int nw, nk, nh, nz, k12_off;
  double w_tail, k12_tail, hs_tail, tz_tail;
  double gam, kx, ky, g1x, gmax, hz, tk, zi_sum, zb;
};

// FSK time-split F1 (fsk_kernels.hip FS1-FS3):
// each filtfilt pass of both tones cut into chunks of L outputs, one lane per
// (chunk, tone), every chunk started w samples early from a zero state.  Its
// band-pass output is within kappa * peak|ext x| of scipy's, so each envelope
// is within (kAmbTau + tau_env) * peak of the reference's, tau_env = kappa *
// ||ifft(h)||_1 (scipy.signal.hilbert's kernel), and F2 flags with that
// margin instead of kAmbTau's; flagged streams re-run the serial F1 (E1).
struct FskSplit {
  int64_t L;                  // outputs per chunk
  int64_t w;                  // warm-up samples (both passes, both tones)
  int64_t c;                  // chunks per pass: ceil(m1 / L), m1 = n + 2 pad
  double tau;                 // kAmbTau + tau_env: F2's margin scale for these streams
  double* y1;                 // [B][2][m1] forward outputs (tone-major per stream)
  unsigned long long* peak;   // [B] bits of max |ext x| (cleared per launch)
  // chunk start states by convolution (FS0, as the PSK split's KS0): conv = 1 uses them
  int conv;
  const double* ktab;         // [2 tones][w][6] (iir_design.h split_state_tables)
  const double* z0tab;        // [2 tones][w + 1][6]
  double* zs;                 // [B][2][c][6] start states, FS0 -> FS1 (then reused for FS2)
  // STRICT (round 6; split_strict.h strict_design_bp per tone, fsk_kernels.hip
  // FS0-FS2 with ST, KF1-KF2, FS3): F2's margin from a bound on |z_split -
  // z_serial| that holds for every input, in place of kappa * peak
  int strict;
  StrictBp sb[2];             // the per-tone design (device tables + constants)
  double u2;
  double hl1;                 // ||ifft(h)||_1 of scipy.signal.hilbert's kernel at n
  unsigned long long* bnd;    // [B][2][8] bits: D1max, E1max, max|y1|, D2max, S1max, -, Fmax, -
  double* sc;                 // [B][2][sstride]: d1 nb1 | d2 nb1 | ds1 c | ds2 c | e1 nb1 | s1 nb1 | e2 nb1
  int64_t sstride, nb1;
};
__host__ __device__ inline int64_t fsk_strict_off_d2(const FskSplit& s) { return s.nb1; }
__host__ __device__ inline int64_t fsk_strict_off_ds1(const FskSplit& s) { return 2 * s.nb1; }
__host__ __device__ inline int64_t fsk_strict_off_ds2(const FskSplit& s) { return 2 * s.nb1 + s.c; }
__host__ __device__ inline int64_t fsk_strict_off_e1(const FskSplit& s) { return 2 * s.nb1 + 2 * s.c; }
__host__ __device__ inline int64_t fsk_strict_off_s1(const FskSplit& s) { return 3 * s.nb1 + 2 * s.c; }
__host__ __device__ inline int64_t fsk_strict_off_e2(const FskSplit& s) { return 4 * s.nb1 + 2 * s.c; }

struct FskIir {            // [tone][tap], tone 0 = mark
  double b[2][8];
  double a[2][8];
  double zi[2][8];
};

// Transmit side (tx_kernels.hip / tx_api.cpp): scalars of one modulate call.
struct TxParams {
  int mode;              // AMR_TX_*
  int64_t sps;           // samples per symbol (per bit for FSK)
  int64_t ramp;          // int(sps * 0.1)          (PSK envelope)
  int64_t n_out;         // samples written per stream
  int64_t sym_stride;    // phases kept per stream = ceil(n_out / sps)
  double c0, c1;         // 2*pi*f0, 2*pi*f1
  double fs;             // sample rate
  double inc0, inc1;     // CPFSK phase increments (bit 1 = f0 = mark, bit 0 = f1 = space)
};

}  // namespace amr
