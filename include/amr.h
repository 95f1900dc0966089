/*
 * amr.h -- C ABI of libamr.so, the MI355X (gfx950) batched demodulator core.
 *
 * Plain C: pointers, sizes and status codes only.  Host-side callers are the
 * drop-in Python modules in audio-modem-radio_amd/ (ctypes; INTEGRATION.md
 * shows the binding) and bench.py.
 *
 * Each entry point names the reference interface it replaces
 * (paths relative to szumanski/Audio-Modem-Radio):
 *
 *   amr_psk_plan_create     the per-call filter/LO setup inside
 *                           modem.qpsk_demodulate   modem.py:191-204
 *                           modem.bpsk_demodulate   modem.py:70-88
 *                           (the host designs b/a/zi with scipy exactly like
 *                            the reference and hands them over; the LO table
 *                            is numpy's exp(-1j*2*pi*fc*t), modem.py:82,201)
 *   amr_psk_demod_host      modem.qpsk_demodulate(samples, baud, carrier, fs)
 *                           modem.py:189-266 (also psk8_demodulate modem.py:348,
 *                           ofdm_demodulate_simple modem.py:375-376, and the
 *                           decoder dispatch decoder.py:422-434) and
 *                           modem.bpsk_demodulate modem.py:68-135 -- for a whole
 *                           batch of equal-length streams per call
 *   amr_psk_demod_device    the same with the batch already resident in HBM
 *   amr_psk_demod_host_edges  the same for a raw-integer / float16 array, whose
 *                           odd extension scipy forms in that dtype (modem.py:198, 77)
 *   amr_psk_demod_fec_device  8PSK alias + fec.ReedSolomonFEC.decode fused
 *                           (modem.py:348 then fec.py:34-69; BASELINE config 5)
 *   amr_fsk_plan_create     the per-call butter/lfilter_zi setup of
 *                           modem.fsk_demodulate    modem.py:301-307
 *   amr_fsk_demod_host      modem.fsk_demodulate    modem.py:298-341 (also
 *                           fsk_high_speed_demodulate modem.py:355-356,
 *                           ft8_demodulate modem.py:391), batched
 *   amr_fsk_envelopes_host  the envelopes |hilbert(filtfilt(.))| modem.py:308-309
 *   amr_hilbert_host        scipy.signal.hilbert as modem.py:309 calls it
 *   amr_resample_host       scipy.signal.resample in decode_wav_file decoder.py:385-387
 *   amr_fec_decode_host     fec.ReedSolomonFEC.decode  fec.py:34-69, batched
 *   amr_frame_parse_host    decoder.parse_fbp_stream_enhanced  decoder.py:142-208,
 *                           batched (magic search, checks, payload CRC32)
 *   amr_modulate_host       modem.bpsk_modulate / qpsk_modulate / fsk_modulate
 *                           (modem.py:28-65, 138-186, 270-295) + the int16 of
 *                           wav_from_array (modem.py:360-368), batched
 *   amr_allgather           the gather of decoded bytes across GPUs (RCCL)
 *
 * Status: every function returns AMR_OK (0) or a negative AMR_E_* code;
 * amr_last_error() gives the message of the calling thread's last failure.
 * Ownership: host buffers are borrowed for the duration of a synchronous
 * call; device buffers passed to *_device calls must stay valid until the
 * plan's stream is synchronised (amr_psk_plan_synchronize).  A plan owns its
 * device scratch; calls on one plan are serialised by a per-plan mutex, so
 * two host threads may share a plan (the reference decodes from a capture
 * QThread and the GUI thread, filebeep_advanced_v2.py:324,1112).
 */
#ifndef AMR_H
#define AMR_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define AMR_ABI_VERSION 5   /* 2: AMR_TF_EXACT (AMR_TF_COUNT 5), amr_fsk_plan_exact_streams / _set_exact_mode,
                                 amr_resample_host bit-exact; size timing arrays from AMR_*_COUNT
                               3: AMR_LAYOUT_SPLIT, amr_psk_plan_set_layout, amr_psk_plan_split_info,
                                  amr_psk_split_design, amr_psk_split_symbols_host, the float32 hand-off
                                  (amr_psk_f32_margin, amr_psk_plan_last_f32f), amr_fsk_plan_resident_bytes,
                                  the FSK time-split F1 (AMR_FSK_LAYOUT_*, amr_fsk_plan_set_layout,
                                  amr_fsk_plan_split_info, amr_fsk_split_design, amr_fsk_split_bandpass_host)
                               4: the time-split passes' chunk start states by convolution
                                  (amr_split_state_tables, amr_psk_plan_split_conv, amr_fsk_plan_split_conv)
                               5: raw-integer captures: amr_psk_demod_host_edges / _device_edges,
                                  amr_fsk_demod_host_edges / _device_edges (the odd extension as the
                                  caller's dtype forms it); the PSK split's strict mode
                                  (amr_psk_plan_set_split_strict ...); F2's margin from a standard
                                  FFT rounding bound (amr_fsk_fft_margin, amr_fsk_plan_margin); the FSK
                                  split's strict mode (amr_fsk_plan_set_split_strict ...) */

#define AMR_OK 0
#define AMR_E_INVALID -1      /* bad argument */
#define AMR_E_PADLEN -2       /* n_samples <= filtfilt padlen (scipy ValueError) */
#define AMR_E_HIP -3          /* HIP runtime failure (message in amr_last_error) */
#define AMR_E_NOMEM -4        /* device allocation failed */
#define AMR_E_NODEVICE -5     /* no usable gfx950 device */
#define AMR_E_RCCL -6         /* RCCL failure */
#define AMR_E_CAPACITY -7     /* batch larger than the plan's max_streams */

#define AMR_DTYPE_F32 0       /* float32 samples (live capture path) */
#define AMR_DTYPE_F64 1       /* float64 samples (decode_wav_file path) */
#define AMR_DTYPE_I16 2       /* int16 PCM, read as int16/32768.0 (libsndfile default) */

#define AMR_PSK_QPSK 0        /* DQPSK slicer, modem.py:216-241 */
#define AMR_PSK_BPSK 1        /* DBPSK slicer, modem.py:102-105 */

/* kernel timing slots reported by amr_psk_plan_timings() */
#define AMR_T_BANDPASS 0
#define AMR_T_LOWPASS_FWD 1
#define AMR_T_LOWPASS_BWD 2
#define AMR_T_LOWPASS_EXACT 3
#define AMR_T_SYNC_PACK 4
#define AMR_T_FEC 5
#define AMR_T_LAUNCH 6     /* the whole launch: first kernel start -> last output written, or, when the
                            * launch's outputs are all-gathered (amr_allgather with this plan), -> gathered */
#define AMR_T_COUNT 7

typedef struct amr_psk_plan amr_psk_plan;
typedef struct amr_comm amr_comm;

int amr_abi_version(void);
/* sha256 prefix of the sources this library was built from (build.py
 * source_hash): ties a loaded binary to the tree's sources */
const char *amr_build_id(void);
const char *amr_last_error(void);
int amr_device_count(int *count);

/* ---- memory helpers (device = the plan's / current device) ---------------- */
int amr_set_device(int device);
int amr_malloc(void **dptr, int64_t bytes);
int amr_free(void *dptr);
int amr_memcpy_h2d(void *dst, const void *src, int64_t bytes);
int amr_memcpy_d2h(void *dst, const void *src, int64_t bytes);
int amr_memcpy_d2d(void *dst, const void *src, int64_t bytes);
int amr_device_synchronize(void);

/* ---- DPSK demodulation ------------------------------------------------------
 * kind          AMR_PSK_QPSK | AMR_PSK_BPSK
 * n_samples     samples per stream (all streams of a call share it)
 * sps           int(fs / baud)                                 modem.py:70,191
 * first_symbol  sps // 2 (QPSK, modem.py:209) or sps (BPSK, modem.py:92)
 * bp_*          band-pass b, a, lfilter_zi (ntaps each; a[0] must be 1)
 * lp_*          low-pass  b, a, lfilter_zi
 * lo4           [n_samples][4] doubles: lo_re, lo_im, -(0*lo_im), 0*lo_re
 *               where lo = numpy.exp(-1j*2*pi*carrier*arange(n)/fs)
 * max_streams   largest batch this plan will see (sizes the HBM scratch)
 */
int amr_psk_plan_create(amr_psk_plan **plan, int device, int kind, int64_t n_samples, int64_t sps,
                        int64_t first_symbol, const double *bp_b, const double *bp_a, const double *bp_zi,
                        int bp_ntaps, const double *lp_b, const double *lp_a, const double *lp_zi,
                        int lp_ntaps, const double *lo4, int64_t max_streams);
int amr_psk_plan_destroy(amr_psk_plan *plan);
/* bytes a stream's output can need: floor(bits/8) */
int64_t amr_psk_plan_out_capacity(const amr_psk_plan *plan);
/* the most device memory the plan can hold: scratch (its row-layout buffers
 * are allocated on the first call that runs that layout) + the host-API
 * staging (allocated on the first amr_psk_demod_host call) */
int64_t amr_psk_plan_scratch_bytes(const amr_psk_plan *plan);
/* the amr_psk_plan_scratch_bytes a plan of this shape would report, without
 * creating it (the drop-in plan cache evicts for it first); < 0 on bad args */
int64_t amr_psk_plan_bytes_estimate(int kind, int64_t n_samples, int64_t sps, int64_t first, int bp_ntaps,
                                    int lp_ntaps, int64_t max_streams);
int amr_psk_plan_synchronize(amr_psk_plan *plan);
/* record per-kernel HIP events on the plan's stream (1) or not (0) */
int amr_psk_plan_enable_timing(amr_psk_plan *plan, int on);
/* hint: the caller keeps `batches` batches in flight at once, each on its own
 * plan (stream); the band-pass layout is then chosen for n_streams x batches
 * concurrent streams.  Default 1.  No reference counterpart:
 * a batching knob of this build (the reference decodes one stream per call,
 * decoder.py:417-464). */
int amr_psk_plan_set_inflight(amr_psk_plan *plan, int batches);
/* milliseconds of each AMR_T_* kernel in the last call (-1 = not run) */
int amr_psk_plan_timings(amr_psk_plan *plan, float *ms, int count);
/* kernel layout of the last call: AMR_LAYOUT_ROW = states spread over lanes
 * (psk_kernels.hip), AMR_LAYOUT_LANE = one stream per lane
 * (psk_lane_kernels.hip), AMR_LAYOUT_SPLIT = each filtfilt pass cut in time
 * into chunks, decisions kept where a margin proves them the reference's and
 * a batch with any other stream re-run by the row kernels
 * (psk_split_kernels.hip).  Picked by streams in flight
 * (DESIGN.md §3): split for <= 64 (one capture at a time, as the reference's
 * own callers decode -- filebeep_advanced_v2.py:324, 1112), row up to
 * 16383, lane from 16384. */
#define AMR_LAYOUT_ROW 0
#define AMR_LAYOUT_LANE 1
#define AMR_LAYOUT_SPLIT 2
int amr_psk_plan_last_layout(const amr_psk_plan *plan);
/* force a layout for this plan's calls (-1: by streams in flight, the
 * default).  No reference counterpart: a test / tuning knob; the bytes are
 * the reference's in every layout. */
int amr_psk_plan_set_layout(amr_psk_plan *plan, int layout);
/* the time-split layout of this plan: streams its last call flagged for the
 * serial path (-1 when that call ran another layout; synchronises the plan's
 * stream), the band-pass / low-pass warm-up samples and the symbols' error
 * bound per unit input peak (-1 when the plan's filters do not allow the
 * layout), and the last call's chunk length (0 before any).  Any pointer may
 * be NULL. */
int amr_psk_plan_split_info(amr_psk_plan *plan, int64_t *flagged, int64_t *warmup_bp, int64_t *warmup_lp,
                            int64_t *chunk, double *kappa);
/* The time-split design of a band-pass / low-pass pair (host arithmetic, no
 * device): warm-up samples per filter and kappa, the bound on a symbol
 * sample's error per unit input peak; AMR_E_INVALID when the
 * filters do not allow the layout (warm-ups over n / 4, not 9 + 5 taps). */
int amr_psk_split_design(const double *bp_b, const double *bp_a, int bp_ntaps, const double *lp_b,
                         const double *lp_a, int lp_ntaps, int64_t n_samples, int64_t n_sym, int64_t *warmup_bp,
                         int64_t *warmup_lp, double *kappa);
/* The lane layout's float32 hand-off: the bound on a symbol
 * sample's error per unit of the stream's max |band-pass output| when the
 * low-pass reads that output rounded to float32 (host arithmetic on the
 * low-pass b, a; 0: no hand-off for these coefficients), and whether the
 * plan's last call used the hand-off (1) or float64 (0). */
double amr_psk_f32_margin(const double *lp_b, const double *lp_a, int lp_ntaps);
int amr_psk_plan_last_f32f(const amr_psk_plan *plan);
/* Diagnostic (tests): the time-split passes alone over a host batch, chunk
 * outputs per lane (0: the plan's rule) -> the symbol samples
 * sym [n_streams][n_sym][re, im] (baseband[first::sps], modem.py:92, 209, as
 * the time-split layout computes them -- not bit-exact).
 * With the convolution chunk starts on, a chunk in 1..127 is refused
 * (AMR_E_INVALID): the start states take n_streams x m1 / chunk x 64 B. */
int amr_psk_split_symbols_host(amr_psk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                               int64_t chunk, double *sym);
/* The time-split band-pass's chunk start states: instead of
 * running w samples of recursion from a zero state, a chunk starting at
 * output t0 takes Z0[t0] v0 + sum_{m < min(t0, w)} K[m] v(t0 - 1 - m) (the
 * Z0 term while t0 <= w), a dot product the GPU spreads over a wave.  Host
 * arithmetic (long double, rounded once) for a DF-II-T filter b, a (a[0] = 1,
 * ntaps - 1 states) and scipy's zi: K [w][ntaps - 1] = the state after a unit
 * input and m zero inputs, Z0 [w + 1][ntaps - 1] = zi after t zero inputs.
 * amr_psk_plan_split_conv: 1 when the plan's time-split layout uses them (its
 * tables are built with the design; AMR_PSK_SPLIT_CONV=0 selects the
 * warm-ups), 0 when not, -1 for NULL.  Both replace no reference function
 * (modem.py:194-199's filtfilt is what they approximate). */
int amr_split_state_tables(const double *b, const double *a, const double *zi, int ntaps, int64_t w, double *K,
                           double *Z0);
int amr_psk_plan_split_conv(amr_psk_plan *plan);
/* The time-split layout's STRICT mode (csrc/split_strict.h).
 * By default a split decision is kept when it clears kappa * peak|x| -- a
 * measured premise (the worst error over the test signal classes and the
 * adversarial search is >= 54x below it), not a bound.  Strict mode keeps it
 * only when it clears a bound that holds for every input: per-step rounding
 * bounds and chunk-start error bounds the kernels measure on the stream itself,
 * carried through the filters' L1 response gains to a bound per symbol; a
 * decision inside it goes to the serial row kernels as before.  Bytes are the
 * reference's in both modes wherever the premise holds; strict mode makes
 * that unconditional at the cost of more flagged captures.
 * amr_psk_plan_set_split_strict: 1 on, 0 off, -1 the process default
 * (AMR_PSK_SPLIT_STRICT=1 turns it on); amr_psk_plan_split_strict: whether this
 * plan's split calls use it; amr_psk_plan_last_strict: whether the last split
 * call did.  No reference counterpart (modem.py:197-214 is what is bounded). */
int amr_psk_plan_set_split_strict(amr_psk_plan *plan, int mode);
int amr_psk_plan_split_strict(amr_psk_plan *plan);
int amr_psk_plan_last_strict(const amr_psk_plan *plan);
/* Diagnostic (tests): the strict passes over a host batch -> the symbol
 * samples sym [n_streams][n_sym][re, im], the bound e [n_streams][n_sym] on
 * each symbol component's |split - reference| and, per stream, scalars
 * [n_streams][4]: E1 (band-pass forward), F (band-pass output), X (mixer
 * output) and P3 (low-pass input peak; negative when the a-posteriori caps
 * failed and the stream would be flagged). */
int amr_psk_split_bounds_host(amr_psk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                              double *sym, double *ebound, double *scalars);
/* The strict design from the filters alone (host arithmetic; the tests'
 * restatement of the bound uses it): consts[32] = g1x, gmax, hz, tk, zi_sum,
 * zb, kx, ky, u2, gam, c3, w1, w2, n_sym, and the sizes nw, nk, nh, ng, nz,
 * k12_off, the cut remainders w_tail, k12_tail, hs_tail, tz_tail, lp_tail,
 * lp_rad, ok, kappa; tabs (NULL: not written) = kabs [w1] | z0abs [w1 + 1] |
 * lpc [n_sym] | W [nw] | K12 [nk] | HS [nh] | GS [ng] | TZ [nz]. */
int amr_psk_split_strict_design(const double *bp_b, const double *bp_a, const double *bp_zi, int bp_ntaps,
                                const double *lp_b, const double *lp_a, const double *lp_zi, int lp_ntaps,
                                int64_t n_samples, int64_t first, int64_t sps, double *consts, double *tabs);
/* number of streams the exact complex low-pass path re-ran in the last call
 * (time-split layout: 0 when no stream was flagged -- the gated row kernels
 * did not run -- else the flagged streams of the row fallback's low-pass) */
int amr_psk_plan_exact_streams(amr_psk_plan *plan, int64_t *count);

/* x: [n_streams][x_stride] samples of `dtype`; out: [n_streams][out_stride]
 * bytes; out_len[s] = bytes written for stream s; sync_idx[s] = bit index of
 * the "FB" sync or -1.  Synchronous. */
int amr_psk_demod_host(amr_psk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                       uint8_t *out, int64_t out_stride, int64_t *out_len, int64_t *sync_idx);
/* Same contract, all pointers device pointers; asynchronous on the plan's stream. */
int amr_psk_demod_device(amr_psk_plan *plan, const void *d_x, int dtype, int64_t n_streams, int64_t x_stride,
                         uint8_t *d_out, int64_t out_stride, int64_t *d_out_len, int64_t *d_sync_idx);
/* Raw-integer captures (ABI 5).  qpsk_demodulate / bpsk_demodulate
 * (modem.py:189-266 / 68-135) hand the caller's array straight to
 * scipy.signal.filtfilt (modem.py:198 / 77), which forms its odd extension
 * 2*x[0] - x[k] (scipy _arraytools.odd_ext, padlen = 3 * bp_ntaps) in the
 * ARRAY's dtype: an int16 capture with |x[0]| > 16383 wraps, uint8 wraps below
 * zero, float16 rounds to half.  A caller with such an array passes the
 * samples converted exactly to AMR_DTYPE_F32 / F64 (their values, not PCM
 * scaling) and the extension as its dtype formed it, in float64:
 *   edges [n_streams][2 * pad]   pad = 3 * bp_ntaps of amr_psk_plan_create
 *   edges[s][j]       = ext index j,           j < pad:  2*x[0] - x[pad - j]
 *   edges[s][pad + r] = ext index pad + n + r, r < pad:  2*x[n-1] - x[n-2-r]
 * (the drop-in builds it with numpy itself, audio-modem-radio_amd/modem.py
 * _raw_input).  Every layout reads the table in place of forming the
 * extension; otherwise as amr_psk_demod_host / _device. */
int amr_psk_demod_host_edges(amr_psk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                             const double *edges, uint8_t *out, int64_t out_stride, int64_t *out_len,
                             int64_t *sync_idx);
int amr_psk_demod_device_edges(amr_psk_plan *plan, const void *d_x, int dtype, int64_t n_streams, int64_t x_stride,
                               const double *d_edges, uint8_t *d_out, int64_t out_stride, int64_t *d_out_len,
                               int64_t *d_sync_idx);
/* qpsk_demodulate / bpsk_demodulate (modem.py:189-266 / 68-135) for a batch,
 * as amr_psk_demod_host, queued on the plan's stream (upload, demod, download)
 * without waiting -- the live-capture loop (filebeep_advanced_v2.py:306-324); the host buffers must stay untouched until amr_psk_plan_synchronize.
 * With two or more plans used in turn, batch k+1's upload overlaps batch k's
 * demod (a stream of batches runs at the PCIe rate).  Page-locked buffers
 * (amr_host_register) make the copies fully asynchronous. */
int amr_psk_demod_host_async(amr_psk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                             uint8_t *out, int64_t out_stride, int64_t *out_len, int64_t *sync_idx);
/* (no reference counterpart: the reference's capture buffers are numpy
 * arrays, sounddevice's callback at filebeep_advanced_v2.py:306)
 * page-locked host memory for capture buffers (hipHostMalloc: the full PCIe
 * rate, 57.6 GB/s measured on the MI355X box, against 38 GB/s for a
 * registered pageable buffer) */
int amr_host_alloc(void **ptr, int64_t bytes);
int amr_host_free(void *ptr);
/* page-lock / release a caller's existing host buffer (hipHostRegister) */
int amr_host_register(void *ptr, int64_t bytes);
int amr_host_unregister(void *ptr);
/* Demod then FEC decode of each stream's bytes, fused on the device. */
int amr_psk_demod_fec_device(amr_psk_plan *plan, const void *d_x, int dtype, int64_t n_streams,
                             int64_t x_stride, uint8_t *d_out, int64_t out_stride, int64_t *d_out_len,
                             int64_t *d_sync_idx, uint8_t *d_fec, int64_t fec_stride, int64_t *d_fec_len,
                             int32_t *d_crc_ok);

/* The slicer stage alone (K4a): differential product s[k+1]*conj(s[k])
 * (modem.py:214 / 100) and the QPSK sector / BPSK sign decision
 * (modem.py:216-241 / 102-105) of sym [n_streams][n_sym] complex doubles
 * (re, im interleaved) -> words [n_streams][ceil(bits/32)], bits MSB first,
 * bits = (n_sym-1)*2 (QPSK) or n_sym-1 (BPSK).  Synchronous, current device.
 * For testing the decision at sector edges directly. */
int amr_psk_slice_host(int kind, const double *sym, int64_t n_streams, int64_t n_sym, uint32_t *words);

/* ---- FSK demodulation (modem.py:298-341) ------------------------------------
 * Replaces modem.fsk_demodulate(samples, baud, mark, space, fs) for a batch of
 * equal-length streams (also fsk_high_speed_demodulate modem.py:355-356,
 * ft8_demodulate modem.py:391 and the decoder's FSK dispatch decoder.py:426-432).
 * n_samples     samples per stream
 * sps           int(fs / baud)                                  modem.py:301
 * mark_* space_* butter(3, [(f-baud)/nyq, (f+baud)/nyq], 'band') b, a and
 *               lfilter_zi (ntaps each, a[0] == 1)              modem.py:307
 * The envelopes |hilbert(filtfilt(...))| (modem.py:308-309) use a double-precision
 * FFT of length n_samples (mixed radix 2/3/4/5, Bluestein otherwise); a stream
 * with a compare the two envelopes' rounding could flip is recomputed exactly
 * (scipy's filtfilt order, pocketfft's transforms), so the decided bytes are
 * the reference's at every length.
 */
#define AMR_TF_BANDPASS 0     /* both tones' filtfilt */
#define AMR_TF_HILBERT 1      /* FFT, -i*sgn(k), inverse FFT, both envelopes and the compare */
#define AMR_TF_DECIDE 2       /* window majority, sync and pack */
#define AMR_TF_LAUNCH 3       /* the whole launch (-> gathered with amr_fsk_allgather), as AMR_T_LAUNCH */
#define AMR_TF_EXACT 4        /* the exact path over the streams F2 flagged (list, filtfilt, envelopes, bits) */
#define AMR_TF_COUNT 5

typedef struct amr_fsk_plan amr_fsk_plan;

int amr_fsk_plan_create(amr_fsk_plan **plan, int device, int64_t n_samples, int64_t sps, const double *mark_b,
                        const double *mark_a, const double *mark_zi, const double *space_b, const double *space_a,
                        const double *space_zi, int ntaps, int64_t max_streams);
int amr_fsk_plan_destroy(amr_fsk_plan *plan);
int64_t amr_fsk_plan_out_capacity(const amr_fsk_plan *plan);
int64_t amr_fsk_plan_scratch_bytes(const amr_fsk_plan *plan);
/* device bytes the plan holds now: scratch_bytes less what the host entries
   allocate on their first call (input / output staging; on a live-layout plan
   the buffer that keeps z through F2) -- a device-entry-only plan's footprint */
int64_t amr_fsk_plan_resident_bytes(const amr_fsk_plan *plan);
/* the amr_fsk_plan_scratch_bytes a plan of this shape would report, without creating it */
int64_t amr_fsk_plan_bytes_estimate(int64_t n_samples, int64_t sps, int ntaps, int64_t max_streams);
/* FFT length actually run: n_samples, or the Bluestein length when n is not 5-smooth */
int64_t amr_fsk_plan_fft_length(const amr_fsk_plan *plan);
/* 1: the plan keeps z and the Hilbert filter's intermediates only for the
 * samples fsk_demodulate's decision windows read (modem.py:320-321: the
 * "live" columns of the four-step grid); 0: every sample */
int amr_fsk_plan_live_columns(const amr_fsk_plan *plan);
int amr_fsk_plan_synchronize(amr_fsk_plan *plan);
int amr_fsk_plan_enable_timing(amr_fsk_plan *plan, int on);
/* the exact path: 0 off (the fast path's bits everywhere -- a diagnostic; decided
 * bytes may then differ from the reference where F2 would have flagged), 1 the
 * streams F2 flags (the default), 2 every stream (tests, timing) */
int amr_fsk_plan_set_exact_mode(amr_fsk_plan *plan, int mode);
/* number of streams the exact path recomputed in the last call (synchronises the plan's stream) */
int amr_fsk_plan_exact_streams(amr_fsk_plan *plan, int64_t *count);
/* milliseconds of each AMR_TF_* stage in the last call (-1 = not run) */
int amr_fsk_plan_timings(amr_fsk_plan *plan, float *ms, int count);
/* Same contracts as amr_psk_demod_host / _device. */
int amr_fsk_demod_host(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                       uint8_t *out, int64_t out_stride, int64_t *out_len, int64_t *sync_idx);
int amr_fsk_demod_device(amr_fsk_plan *plan, const void *d_x, int dtype, int64_t n_streams, int64_t x_stride,
                         uint8_t *d_out, int64_t out_stride, int64_t *d_out_len, int64_t *d_sync_idx);
/* fsk_demodulate's raw-integer captures (modem.py:308 filtfilt on the
 * caller's array): as amr_psk_demod_host_edges, pad = 3 * ntaps of
 * amr_fsk_plan_create (both tones' filters see the same extension).  F2's
 * ambiguity margin then scales with max(peak|x|, peak|edges|). */
int amr_fsk_demod_host_edges(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                             const double *edges, uint8_t *out, int64_t out_stride, int64_t *out_len,
                             int64_t *sync_idx);
int amr_fsk_demod_device_edges(amr_fsk_plan *plan, const void *d_x, int dtype, int64_t n_streams, int64_t x_stride,
                               const double *d_edges, uint8_t *d_out, int64_t out_stride, int64_t *d_out_len,
                               int64_t *d_sync_idx);
/* fsk_demodulate (modem.py:298-341), queued without waiting: as
 * amr_psk_demod_host_async */
int amr_fsk_demod_host_async(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                             uint8_t *out, int64_t out_stride, int64_t *out_len, int64_t *sync_idx);
/* mark_env, space_env: [n_streams][n_samples] doubles, |hilbert(filtfilt(.))|
 * of each tone (modem.py:308-309) -- the intermediate the tolerance tests read. */
int amr_fsk_envelopes_host(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                           double *mark_env, double *space_env);
/* F1's layout per call.  SERIAL: scipy's filtfilt, one recursion per (stream,
 * tone).  SPLIT: each filtfilt pass cut in time into chunks started early from
 * a zero state (the latency path of one capture): its band-pass
 * output is within kappa * peak|ext x| of scipy's, F2 flags every compare
 * within (2^-36 + kappa * ||hilbert kernel||_1) * peak of a tie, and the exact
 * path re-runs the serial F1 for those streams -- decided bytes unchanged.
 * AUTO (the default): SPLIT for calls of at most 1024 streams when the plan's
 * filters allow it (warm-up <= n / 4) and the exact path is on. */
#define AMR_FSK_LAYOUT_AUTO 0
#define AMR_FSK_LAYOUT_SERIAL 1
#define AMR_FSK_LAYOUT_SPLIT 2
/* 1 when the plan's time-split F1 starts its chunks from convolution states
 * (FS0, amr_split_state_tables per tone) rather than warm-ups
 * (AMR_FSK_SPLIT_CONV=0), 0 when not (or no split design), -1 for NULL. */
int amr_fsk_plan_split_conv(amr_fsk_plan *plan);
int amr_fsk_plan_set_layout(amr_fsk_plan *plan, int layout);
/* the last call's F1 (*last_split 1: split) and the plan's split design:
 * warm-up samples, chunk length of the last split call, kappa, and tau (F2's
 * margin scale for split calls).  Any pointer may be NULL; *warmup = -1 when
 * the plan cannot split. */
int amr_fsk_plan_split_info(amr_fsk_plan *plan, int *last_split, int64_t *warmup, int64_t *chunk,
                            double *kappa, double *tau);
/* F2's margin scale tau from a standard FFT rounding bound (DESIGN.md §2 item
 * 6; host arithmetic, no device): out[8] = tau (max(2^-36, the bound)), the
 * fast path's and pocketfft's relative 2-norm transform errors eps_fast /
 * eps_ref, the bound on max ||z||_2 / peak|ext x| over both tones, whether
 * the fast path runs Bluestein and its length, whether pocketfft does and its
 * length.  The filters as amr_fsk_plan_create takes them. */
int amr_fsk_fft_margin(int64_t n_samples, const double *mark_b, const double *mark_a, const double *mark_zi,
                       const double *space_b, const double *space_a, const double *space_zi, int ntaps, double *out);
/* a plan's F2 margin scales: tau (serial F1) and tau_split (time-split F1:
 * tau + kappa ||ifft(h)||_1) */
int amr_fsk_plan_margin(amr_fsk_plan *plan, double *tau, double *tau_split);
/* the split design from the filters alone (host arithmetic; no device):
 * warm-up, kappa and ||ifft(h)||_1 of scipy.signal.hilbert's multiplier h at
 * length n.  Returns AMR_E_INVALID when the filters cannot be split at n. */
int amr_fsk_split_design(int64_t n_samples, const double *mark_b, const double *mark_a, const double *space_b,
                         const double *space_a, int ntaps, int64_t *warmup, double *kappa, double *hilbert_l1);
/* The FSK split F1's STRICT mode (fsk_kernels.hip FS0-FS2 with
 * their step bounds, KF1-KF2): F2's margin for a split call becomes tau +
 * F ||ifft(h)||_1 / peak with F a bound on |z_split - z_serial| per tone that
 * holds for every input (the PSK strict mode's band-pass analysis per tone),
 * instead of tau + kappa ||ifft(h)||_1 (a measured premise).  Set: 1 on, 0
 * off, -1 the process default (AMR_FSK_SPLIT_STRICT=0 / 1).  split_strict:
 * whether this plan's split calls use it; last_strict: whether the last did. */
int amr_fsk_plan_set_split_strict(amr_fsk_plan *plan, int mode);
int amr_fsk_plan_split_strict(amr_fsk_plan *plan);
int amr_fsk_plan_last_strict(amr_fsk_plan *plan);
/* The strict band-pass design of ONE filter (host arithmetic; the tests'
 * restatement reads it): w the plan's warm-up (amr_fsk_split_design), consts
 * [32] in amr_psk_split_strict_design's layout (the low-pass fields 0), tabs
 * (NULL: not written) = kabs [w] | z0abs [w + 1] | W | K12 | HS | GS | TZ. */
int amr_fsk_split_strict_design(const double *b, const double *a, const double *zi, int ntaps, int64_t w,
                                double *consts, double *tabs);
/* Diagnostic (tests): the strict split F1 over a host batch: z_out
 * [n_streams][n_samples][2] (mark, space), bnd_out [n_streams][2][8] the
 * per-tone maxima as doubles (D1max, E1max, max|y1|, D2max, S1max, -, F, -),
 * peak_out [n_streams] max |ext x|.  Synchronous. */
int amr_fsk_split_bounds_host(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                              double *z_out, double *bnd_out, double *peak_out);
/* the split F1's band-pass output itself (a diagnostic the tests compare with
 * the oracle's restatement): out [n_streams][n_samples][2] (mark, space);
 * chunk 0 = the plan's rule (1..127 refused with the convolution starts on,
 * as amr_psk_split_symbols_host).  Synchronous. */
int amr_fsk_split_bandpass_host(amr_fsk_plan *plan, const void *x, int dtype, int64_t n_streams, int64_t x_stride,
                                int64_t chunk, double *out);

/* ---- FFT / Hilbert (the transforms under scipy.signal.hilbert) --------------
 * in/out: [batch][n] interleaved complex doubles; inverse scales by 1/n
 * (numpy.fft.fft / numpy.fft.ifft).  analytic: [batch][n] complex doubles =
 * scipy.signal.hilbert(x) for real x [batch][n].  Synchronous, on `device`. */
int amr_fft_c2c_host(const double *in, double *out, int64_t n, int64_t batch, int inverse, int device);
int amr_hilbert_host(const double *x, double *analytic, int64_t n, int64_t batch, int device);
/* scipy.signal.resample(x, num) of each real row (x: [batch][nx] -> y: [batch][num]),
 * as decoder.decode_wav_file calls it (decoder.py:385-387), bit for bit:
 * pocketfft's rfft (every radix, Bluestein), the reference's spectrum
 * truncation / zero-padding with its Nyquist-bin rule, pocketfft's irfft,
 * times num/nx (pocketfft_dev.h). */
int amr_resample_host(const double *x, int64_t nx, int64_t num, int64_t batch, double *y, int device);
/* |scipy.signal.hilbert(x)| of each real row (x: [batch][n] -> env), evaluated
 * as pocketfft + numpy do, bit for bit (the FSK exact path's envelope stage,
 * modem.py:309; a diagnostic entry for tests) */
int amr_hilbert_env_exact_host(const double *x, int64_t n, int64_t batch, double *env, int device);

/* ---- FEC (fec.py:34-69) -----------------------------------------------------
 * in: [n][in_stride] bytes, in_len[n]; out: [n][out_stride] (>= in_len each);
 * crc_ok[s] = 1 when the recomputed CRC32 equals the trailing word
 * (the reference only prints "Aviso: CRC ..." on mismatch). */
int amr_fec_decode_host(const uint8_t *in, int64_t in_stride, const int64_t *in_len, int64_t n,
                        uint8_t *out, int64_t out_stride, int64_t *out_len, int32_t *crc_ok);

/* ---- FBP frame parse (decoder.py:142-208, parse_fbp_stream_enhanced) --------
 * For every stream's decoded bytes (in: [n][in_stride], in_len[n]): every
 * b'FBPC' occurrence in increasing order, run through the reference's checks
 * in its order, and the CRC32 (binascii.crc32) of the payload of those that
 * pass them.  n_cands[s] = occurrences found (may exceed max_cands: records
 * are kept for the first min(n_cands, max_cands, 256); a caller seeing more
 * parses that stream itself).  recs: [n][max_cands], 1 <= max_cands <=
 * AMR_FRAME_MAX_CANDS (larger is AMR_E_INVALID).  The host turns records
 * into the reference's list of {'name', 'data', 'final_crc'} and log lines. */
#define AMR_FRAME_MAX_CANDS 256     /* records kept per stream (LDS list of k_frame_parse) */
#define AMR_FRAME_SHORT 0          /* start + 30 > len(raw)            decoder.py:165 */
#define AMR_FRAME_NONAME 1         /* name_len == 0                     decoder.py:169 */
#define AMR_FRAME_NOMETA 2         /* meta_start + 24 > len(raw)        decoder.py:177 */
#define AMR_FRAME_BADLEN 3         /* dlen > 50_000_000 or dlen == 0    decoder.py:182 */
#define AMR_FRAME_INCOMPLETE 4     /* payload past the end: "Dados incompletos"  :185-187 */
#define AMR_FRAME_CRC_BAD 5        /* "Erro de CRC"                     decoder.py:197-198 */
#define AMR_FRAME_OK 6             /* CRC valid: appended               decoder.py:190-196 */
#define AMR_FRAME_PENDING_CRC 7    /* internal */
typedef struct amr_frame_rec {
  int64_t start;                   /* index of the magic */
  int64_t name_start;              /* start + 5 */
  int64_t payload_start;           /* meta_start + 24 */
  int32_t status;                  /* AMR_FRAME_* */
  int32_t name_len;                /* raw[start + 4] */
  uint32_t part, total, fsize, fcrc, dlen, pcrc;   /* '<IIIIII' at meta_start */
  uint32_t calc_crc;               /* crc32(payload) when computed */
  uint32_t reserved;
} amr_frame_rec;                   /* 64 bytes */
int amr_frame_parse_host(const uint8_t *in, int64_t in_stride, const int64_t *in_len, int64_t n,
                         int64_t max_cands, int32_t *n_cands, amr_frame_rec *recs);
/* device pointers, enqueued on the plan's stream (plan may be NULL: the null stream) */
int amr_frame_parse_device(amr_psk_plan *plan, const uint8_t *d_in, int64_t in_stride, const int64_t *d_in_len,
                           int64_t n, int64_t max_cands, int32_t *d_n_cands, amr_frame_rec *d_recs);

/* ---- transmit side (modem.py:28-65, 138-186, 270-295, 360-368) ------------
 * The reference's modulators for a batch of payloads: data [n][data_stride]
 * bytes, n_bytes[n].  out [n][out_stride] float32: each stream's waveform
 * (bpsk_modulate / qpsk_modulate / fsk_modulate, sample for sample) cut or
 * zero-padded to n_out samples; pcm (optional, may be NULL) the same samples
 * as modem.wav_from_array writes them, int16(out * 32767).
 * f0 = carrier (PSK) or mark_freq (FSK); f1 = space_freq (FSK only).
 * A PSK symbol of 1..9 samples is the reference's numpy broadcast ValueError
 * (its 10 % ramp is empty, modem.py:58-61 / 181-183): AMR_E_INVALID with the
 * reference's message in amr_last_error(). */
#define AMR_TX_BPSK 0              /* bpsk_modulate  modem.py:28-65   */
#define AMR_TX_QPSK 1              /* qpsk_modulate  modem.py:138-186 */
#define AMR_TX_FSK 2               /* fsk_modulate   modem.py:270-295 */
/* natural waveform length of an n_bytes payload (the reference's len(out)), or < 0 */
int64_t amr_tx_samples(int mode, int64_t n_bytes, double baud, double sample_rate);
/* device scratch bytes amr_modulate_device needs for this shape */
int64_t amr_tx_work_bytes(int mode, double baud, double sample_rate, int64_t n_streams, int64_t n_out);
int amr_modulate_host(int mode, double baud, double f0, double f1, double sample_rate, const uint8_t *data,
                      int64_t data_stride, const int64_t *n_bytes, int64_t n, float *out, int64_t out_stride,
                      int64_t n_out, int16_t *pcm, int64_t pcm_stride);
/* device pointers, enqueued on the plan's stream (plan may be NULL: the null stream) */
int amr_modulate_device(amr_psk_plan *plan, int mode, double baud, double f0, double f1, double sample_rate,
                        const uint8_t *d_data, int64_t data_stride, const int64_t *d_n_bytes, int64_t n,
                        float *d_out, int64_t out_stride, int64_t n_out, int16_t *d_pcm, int64_t pcm_stride,
                        void *d_work, int64_t work_bytes);

/* ---- benchmark / test input generator (no reference counterpart) ----------
 * d_out[s][i] = d_base[(s + row_offset) % n_base][i] + sigma * N(0,1), float32,
 * the deviate hashed from (seed, s, i): distinct noisy batches over the same
 * clean frames, generated in HBM (bench.py's in-flight batches).  Synchronous. */
int amr_synth_tile_noise(const float *d_base, int64_t n_base, int64_t n_samples, float *d_out, int64_t n_streams,
                         int64_t row_offset, float sigma, uint64_t seed);

/* ---- multi-GPU: RCCL over xGMI ----------------------------------------------- */
#define AMR_UNIQUE_ID_BYTES 128
int amr_comm_unique_id(uint8_t *id /* AMR_UNIQUE_ID_BYTES */);
int amr_comm_create(amr_comm **comm, const uint8_t *id, int nranks, int rank, int device);
int amr_comm_destroy(amr_comm *comm);
/* ncclAllGather of bytes_per_rank bytes per rank, on the comm's own stream in
 * call order (safe with several plans in flight); with a plan it is ordered
 * after the plan's queued work, and the plan's later work waits for it before
 * writing any output (its filters overlap the gather); the plan's
 * synchronize waits for it too. */
int amr_allgather(amr_comm *comm, const void *d_send, void *d_recv, int64_t bytes_per_rank,
                  amr_psk_plan *plan);
/* the same, ordered after / before the FSK plan's queued work */
int amr_fsk_allgather(amr_comm *comm, const void *d_send, void *d_recv, int64_t bytes_per_rank,
                      amr_fsk_plan *plan);
int amr_comm_synchronize(amr_comm *comm);
/* Host-memory collectives of the sharded host path (multi.py RcclTransport;
 * decoder.decode_from_buffer_batch with a transport): synchronous, on the
 * comm's stream behind its earlier gathers, through a device staging buffer
 * the comm keeps.  allgather_host: recv = world x bytes_per_rank, rank-major;
 * allreduce_max: values[i] = max over ranks (count doubles, in place); a
 * barrier is allreduce_max of one value. */
int amr_comm_allgather_host(amr_comm *comm, const void *send, void *recv, int64_t bytes_per_rank);
int amr_comm_allreduce_max(amr_comm *comm, double *values, int64_t count);
int amr_comm_world(const amr_comm *comm, int *nranks, int *rank);

#ifdef __cplusplus
}
#endif
#endif /* AMR_H */
