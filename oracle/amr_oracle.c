/*
 * amr_oracle.c -- CPU restatement of the reference demodulator hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  This file is the checker (and the timed CPU
 * baseline, bench.py's cpu_baseline leg).  Only tests/, __graft_entry__.smoke()
 * and bench.py may load it.  The product path (audio-modem-radio_amd/) never
 * links or calls it.
 *
 * It restates, operation for operation, what the reference computes through
 * numpy/scipy for one stream:
 *
 *   scipy.signal.filtfilt(b, a, x)  (padtype='odd', padlen=3*ntaps)
 *     used at modem.py:77,88 (BPSK), modem.py:198,204 (QPSK), modem.py:308 (FSK).
 *     scipy 1.15.3 _signaltools.py filtfilt: odd_ext (_arraytools.py:99-106),
 *     zi = lfilter_zi * ext[0], forward lfilter, zi * y[-1], reverse lfilter.
 *     lfilter's direct-form-II-transposed inner loop, in scipy's order
 *     (no FMA):  y = z0 + b0*x;  z[i] = (z[i+1] + x*b[i+1]) - y*a[i+1];
 *                z[last] = x*b[last] - y*a[last].
 *     The odd extension is evaluated in the INPUT's precision (numpy keeps a
 *     float32 array float32 in `2*x[0] - x[k]`), then promoted to double.
 *   mixer  filtered * exp(-1j*2*pi*fc*t)   modem.py:80-83, 200-201
 *     (the LO table comes from the caller, evaluated with numpy's own exp).
 *   symbol pick baseband[first::sps]        modem.py:92-93 (BPSK first=sps),
 *                                           modem.py:209   (QPSK first=sps//2)
 *   differential product s[1:]*conj(s[:-1])  modem.py:100, 214
 *     numpy 2.2 on AVX-512/FMA3 x86 evaluates complex multiply as
 *       re = fma(ar, br, -(ai*bi)),  im = fma(ar, bi, ai*br)
 *     (measured bit for bit in this container);
 *     restated here with the C99 fma().
 *   QPSK slicer   modem.py:216-241   np.angle, +2pi if negative, 4 sectors.
 *     np.angle is numpy's arctan2, which numpy 2.2 evaluates with its AVX-512
 *     (SVML) kernel on the hosts the golden fixtures came from
 *     (numpy._core.__cpu_features__['AVX512_SKX'], recorded in
 *     tests/golden/manifest.json).  That kernel is not correctly rounded: within
 *     an ulp of a sector edge it differs from libm's atan2 on ~6 % of inputs,
 *     enough to flip a decision.  np_angle() below restates its result there
 *     (numpy_atan2_near_diag) and uses libm elsewhere; tests/test_oracle_slicer.py
 *     checks it against numpy on the sector edges and 1.5 M near-tie pairs.
 *   BPSK slicer   modem.py:102-105   real(diff) < 0 -> 1
 *   sync + pack   modem.py:111-135 (BPSK), 243-266 (QPSK), 326-341 (FSK)
 *     first index of "0100011001000010" at any bit offset; pack MSB first
 *     from there (or from 0 when absent); floor(L/8) bytes.
 *   FEC decode    fec.py:34-69  parity-XOR triples + CRC32 (zlib polynomial)
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off; no -ffast-math).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define AMR_DT_F32 0
#define AMR_DT_F64 1
#define AMR_DT_I16 2      /* int16 PCM read as int16 / 32768 (decode_wav_file's libsndfile data) */
/* Raw samples of the caller's own dtype, as the reference's public functions
 * take them (modem.py:77, 198, 308 hand `samples` straight to filtfilt): the
 * values are the samples themselves, and scipy's odd extension 2*x[0] - x[k]
 * (_arraytools.py odd_ext) is evaluated in THAT dtype's numpy arithmetic --
 * integers wrap modulo 2^bits (2 * an int16 array stays int16 under NEP 50),
 * bool promotes to int64, float16 rounds each operation to half. */
#define AMR_DT_RAW_I8 3
#define AMR_DT_RAW_U8 4
#define AMR_DT_RAW_I16 5
#define AMR_DT_RAW_U16 6
#define AMR_DT_RAW_I32 7
#define AMR_DT_RAW_U32 8
#define AMR_DT_RAW_I64 9
#define AMR_DT_RAW_U64 10
#define AMR_DT_RAW_BOOL 11
#define AMR_DT_F16 12

static size_t dt_size(int dtype)
{
    switch (dtype) {
    case AMR_DT_F32: case AMR_DT_RAW_I32: case AMR_DT_RAW_U32: return 4;
    case AMR_DT_I16: case AMR_DT_RAW_I16: case AMR_DT_RAW_U16: case AMR_DT_F16: return 2;
    case AMR_DT_RAW_I8: case AMR_DT_RAW_U8: case AMR_DT_RAW_BOOL: return 1;
    default: return 8;
    }
}

/* IEEE binary16 <-> binary32, round to nearest even (numpy's npy_half_to_float /
 * npy_float_to_half; numpy's float16 ufuncs compute in float32 and round the
 * result to half, which equals a correctly rounded half operation: 24 >= 2*11+2) */
static float f16_to_f32(uint16_t h)
{
    const uint32_t s = (uint32_t)(h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu;
    uint32_t b;
    float f;
    if (e == 0) { f = ldexpf((float)m, -24); return s ? -f : f; }
    b = e == 31 ? (s | 0x7f800000u | (m << 13)) : (s | ((e + 112u) << 23) | (m << 13));
    memcpy(&f, &b, 4);
    return f;
}
static uint16_t f32_to_f16(float f)
{
    uint32_t b;
    memcpy(&b, &f, 4);
    const uint16_t s = (uint16_t)((b >> 16) & 0x8000u);
    const uint32_t a = b & 0x7fffffffu;
    if (a > 0x7f800000u) return (uint16_t)(s | 0x7e00u | ((a >> 13) & 0x3ffu));   /* NaN */
    if (a >= 0x477ff000u) return (uint16_t)(s | 0x7c00u);         /* >= 65520 (a tie to even: inf) or inf */
    if (a < 0x38800000u) {                                         /* below 2^-14: a subnormal half */
        float v;
        memcpy(&v, &a, 4);
        return (uint16_t)(s | (uint16_t)rintf(v * 16777216.0f)); /* units of 2^-24, exact scaling, RNE */
    }
    uint32_t r = a - 0x38000000u, h = r >> 13, rem = r & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) ++h;
    return (uint16_t)(s | h);
}

/* ---- lfilter (DF-II-T) ----------------------------------------------------
 * scipy/signal lfilter inner loop, real double case.  x and y may alias.   */
static void df2t(const double *b, const double *a, int nt, double *z,
                 const double *x, double *y, int64_t n, int64_t step)
{
    for (int64_t k = 0; k < n; ++k) {
        const double xn = x[k * step];
        const double yn = z[0] + b[0] * xn;
        for (int i = 0; i < nt - 2; ++i)
            z[i] = z[i + 1] + xn * b[i + 1] - yn * a[i + 1];
        z[nt - 2] = xn * b[nt - 1] - yn * a[nt - 1];
        y[k * step] = yn;
    }
}

/* sample i as lfilter sees it: numpy's cast of the array to float64 */
static double load_x(const void *x, int dtype, int64_t i)
{
    switch (dtype) {
    case AMR_DT_F32: return (double)((const float *)x)[i];
    case AMR_DT_I16: return (double)((const int16_t *)x)[i] / 32768.0;
    case AMR_DT_RAW_I8: return (double)((const int8_t *)x)[i];
    case AMR_DT_RAW_U8: return (double)((const uint8_t *)x)[i];
    case AMR_DT_RAW_I16: return (double)((const int16_t *)x)[i];
    case AMR_DT_RAW_U16: return (double)((const uint16_t *)x)[i];
    case AMR_DT_RAW_I32: return (double)((const int32_t *)x)[i];
    case AMR_DT_RAW_U32: return (double)((const uint32_t *)x)[i];
    case AMR_DT_RAW_I64: return (double)((const int64_t *)x)[i];
    case AMR_DT_RAW_U64: return (double)((const uint64_t *)x)[i];
    case AMR_DT_RAW_BOOL: return ((const uint8_t *)x)[i] ? 1.0 : 0.0;
    case AMR_DT_F16: return (double)f16_to_f32(((const uint16_t *)x)[i]);
    default: return ((const double *)x)[i];
    }
}

/* 2*x[e] - x[k] in the dtype's own arithmetic (_arraytools.py:103), then as float64 */
static double odd_pair(const void *x, int dtype, int64_t e, int64_t k)
{
    switch (dtype) {
    case AMR_DT_F32: { const float *v = (const float *)x; return (double)(2.0f * v[e] - v[k]); }
    case AMR_DT_RAW_I8: { const uint8_t *v = (const uint8_t *)x; return (double)(int8_t)(uint8_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_U8: { const uint8_t *v = (const uint8_t *)x; return (double)(uint8_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_I16: {
        const uint16_t *v = (const uint16_t *)x;
        return (double)(int16_t)(uint16_t)(2u * v[e] - v[k]);
    }
    case AMR_DT_RAW_U16: { const uint16_t *v = (const uint16_t *)x; return (double)(uint16_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_I32: { const uint32_t *v = (const uint32_t *)x; return (double)(int32_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_U32: { const uint32_t *v = (const uint32_t *)x; return (double)(uint32_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_I64: { const uint64_t *v = (const uint64_t *)x; return (double)(int64_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_U64: { const uint64_t *v = (const uint64_t *)x; return (double)(uint64_t)(2u * v[e] - v[k]); }
    case AMR_DT_RAW_BOOL: {   /* 2 * bool -> int64 (numpy's default integer), no wrap */
        const uint8_t *v = (const uint8_t *)x;
        return (double)(2 * (int64_t)(v[e] != 0) - (int64_t)(v[k] != 0));
    }
    case AMR_DT_F16: {
        const uint16_t *v = (const uint16_t *)x;
        const uint16_t t = f32_to_f16(2.0f * f16_to_f32(v[e]));
        return (double)f16_to_f32(f32_to_f16(f16_to_f32(t) - f16_to_f32(v[k])));
    }
    default:   /* f64 and the i16 PCM (decode_wav_file hands the demod float64 = i16/32768) */
        return 2.0 * load_x(x, dtype, e) - load_x(x, dtype, k);
    }
}

/* odd extension sample j of the padded sequence (0 <= j < n + 2*pad),
 * evaluated in the input's own dtype as numpy does (_arraytools.py:103). */
static double ext_sample(const void *x, int dtype, int64_t n, int pad, int64_t j)
{
    if (j >= pad && j < pad + n) return load_x(x, dtype, j - pad);
    if (j < pad) return odd_pair(x, dtype, 0, pad - j);
    return odd_pair(x, dtype, n - 1, n - 2 - (j - pad - n));
}

/* The 2*pad extension samples of one stream in libamr.so's edge-table order
 * (include/amr.h amr_psk_demod_host_edges): out[j] = ext index j (the left
 * pad), out[pad + r] = ext index pad + n + r (the right).  The product builds
 * this table with numpy itself; tests check it against this C restatement. */
int oracle_odd_edges(const void *x, int dtype, int64_t n, int pad, double *out)
{
    if (pad < 1 || n <= pad) return -1;
    for (int j = 0; j < pad; ++j) out[j] = ext_sample(x, dtype, n, pad, j);
    for (int r = 0; r < pad; ++r) out[pad + r] = ext_sample(x, dtype, n, pad, pad + n + r);
    return 0;
}

/* scipy.signal.filtfilt(b, a, x) with default odd padding, padlen = 3*nt.
 * work: 2*(n + 2*pad) doubles.  out: n doubles.  Returns -1 if n <= pad. */
int oracle_filtfilt(const double *b, const double *a, int nt, const double *zi,
                    const void *x, int dtype, int64_t n, double *out, double *work)
{
    const int pad = 3 * nt;
    if (n <= pad) return -1;
    const int64_t m = n + 2 * (int64_t)pad;
    double z[32];
    double *ext = work;
    for (int64_t j = 0; j < m; ++j) ext[j] = ext_sample(x, dtype, n, pad, j);
    for (int i = 0; i < nt - 1; ++i) z[i] = zi[i] * ext[0];
    df2t(b, a, nt, z, ext, ext, m, 1);                 /* forward, in place */
    for (int i = 0; i < nt - 1; ++i) z[i] = zi[i] * ext[m - 1];
    df2t(b, a, nt, z, ext + m - 1, ext + m - 1, m, -1); /* backward over reversed */
    for (int64_t i = 0; i < n; ++i) out[i] = ext[pad + i];
    return 0;
}

/* ---- complex filtfilt, exact numpy/scipy semantics --------------------------
 * filtfilt on a complex128 sequence with real coefficients (modem.py:88, 204).
 * scipy's complex lfilter inner loop (CDOUBLE_filt) evaluates every tap
 * product as a complex multiply by (b + 0j) normalised by a0 = 1:
 *     re = (b*xr - (+0)*xi) / 1,   im = ((+0)*xr + b*xi) / 1
 * and numpy builds the odd extension (2*x[0] - x[k]) and zi*x[0] with its
 * complex multiply  re = fma(ar, br, -(ai*bi)), im = fma(ar, bi, ai*br).
 * The extra terms only ever change the SIGN OF A ZERO, but a signed zero
 * reaches np.angle in silent (exactly zero) regions, so the oracle keeps them.
 * Verified bit for bit against scipy.signal.lfilter on signed-zero inputs. */
static void df2t_cplx(const double *b, const double *a, int nt, double *zr, double *zi,
                      double *xr, double *xi, int64_t n, int64_t step)
{
    for (int64_t k = 0; k < n; ++k) {
        const double x0 = xr[k * step], x1 = xi[k * step];
        const double t0x = 0.0 * x1, t1x = 0.0 * x0;
        const double y0 = zr[0] + (b[0] * x0 - t0x);
        const double y1 = zi[0] + (t1x + b[0] * x1);
        const double t0y = 0.0 * y1, t1y = 0.0 * y0;
        int i = 0;
        for (; i < nt - 2; ++i) {
            double r = zr[i + 1] + (b[i + 1] * x0 - t0x);
            double m = zi[i + 1] + (t1x + b[i + 1] * x1);
            zr[i] = r - (a[i + 1] * y0 - t0y);
            zi[i] = m - (t1y + a[i + 1] * y1);
        }
        zr[i] = (b[i + 1] * x0 - t0x) - (a[i + 1] * y0 - t0y);
        zi[i] = (t1x + b[i + 1] * x1) - (t1y + a[i + 1] * y1);
        xr[k * step] = y0;
        xi[k * step] = y1;
    }
}

/* numpy complex multiply (ar + i ai)*(br + i bi) on AVX-512/FMA3 x86 */
static inline void cmul_np(double ar, double ai, double br, double bi, double *re, double *im)
{
    *re = fma(ar, br, -(ai * bi));
    *im = fma(ar, bi, ai * br);
}

static int filtfilt_complex(const double *b, const double *a, int nt, const double *zi,
                            double *re, double *im, int64_t n, double *work)
{
    const int pad = 3 * nt;
    if (n <= pad) return -1;
    const int64_t m = n + 2 * (int64_t)pad;
    double *er = work, *ei = work + m;
    double zr[32], zc[32], tr, ti;
    /* odd extension: 2*x[0] - x[k] as numpy complex ops (_arraytools.py:103) */
    cmul_np(2.0, 0.0, re[0], im[0], &tr, &ti);
    for (int j = 0; j < pad; ++j) { er[j] = tr - re[pad - j]; ei[j] = ti - im[pad - j]; }
    for (int64_t j = 0; j < n; ++j) { er[pad + j] = re[j]; ei[pad + j] = im[j]; }
    cmul_np(2.0, 0.0, re[n - 1], im[n - 1], &tr, &ti);
    for (int j = 0; j < pad; ++j) { er[pad + n + j] = tr - re[n - 2 - j]; ei[pad + n + j] = ti - im[n - 2 - j]; }
    for (int i = 0; i < nt - 1; ++i) cmul_np(zi[i], 0.0, er[0], ei[0], &zr[i], &zc[i]);
    df2t_cplx(b, a, nt, zr, zc, er, ei, m, 1);
    for (int i = 0; i < nt - 1; ++i) cmul_np(zi[i], 0.0, er[m - 1], ei[m - 1], &zr[i], &zc[i]);
    df2t_cplx(b, a, nt, zr, zc, er + m - 1, ei + m - 1, m, -1);
    for (int64_t i = 0; i < n; ++i) { re[i] = er[pad + i]; im[i] = ei[pad + i]; }
    return 0;
}

/* ---- np.angle near a sector edge (modem.py:219) ---------------------------
 * numpy's AVX-512 arctan2 within |t| < 2^-29 of the diagonal |y| = |x|, for
 * components of magnitude 2^-1015 .. 2^985, bit for bit:
 *   t  = (|y| - |x|) / (|y| + |x|)
 *   x > 0:  pi4 + (t + pi4_lo)            x < 0:  pi - (pi4 - (pi_lo - (t + pi4_lo)))
 * negated for y < 0, with pi/4 split into double hi + lo and pi into hi +
 * SVML's short lo 0x1.1a64p-53 (bisecting numpy's rounding boundaries in the
 * pi-side form located exactly this constant, not pi - hi).  Outside that
 * domain (and for zeros / inf / NaN) libm's atan2 is numpy's result on every
 * input the tests cover.  The GPU slicer (psk_common.h) uses the same model. */
static int numpy_atan2_near_diag(double y, double x, double *ang)
{
    const double ay = fabs(y), ax = fabs(x);
    if (!(ax >= 0x1p-1015 && ax <= 0x1p985 && ay >= 0x1p-1015 && ay <= 0x1p985)) return 0;
    const double t = (ay - ax) / (ay + ax);
    if (!(fabs(t) < 0x1p-29)) return 0;
    const double pi4 = 0x1.921fb54442d18p-1, pi4_lo = 0x1.1a62633145c07p-55;
    const double pi = 0x1.921fb54442d18p+1, pi_lo = 0x1.1a64p-53;   // SVML's short pi_lo
    const double a = x > 0 ? pi4 + (t + pi4_lo) : pi - (pi4 - (pi_lo - (t + pi4_lo)));
    *ang = y < 0 ? -a : a;
    return 1;
}

static double np_angle(double re, double im)
{
    double ang;
    if (!numpy_atan2_near_diag(im, re, &ang)) ang = atan2(im, re);
    return ang;
}

/* the reference's sector decision for one differential product (modem.py:219-241):
 * returns the dibit as 2*hi + lo */
static int qpsk_dibit(double dr, double di)
{
    double ang = np_angle(dr, di);                   /* np.angle, modem.py:219 */
    if (ang < 0) ang += 2 * M_PI;                    /* modem.py:232 */
    if (ang < M_PI / 4 || ang > 7 * M_PI / 4) return 0;
    if (M_PI / 4 <= ang && ang < 3 * M_PI / 4) return 1;
    if (3 * M_PI / 4 <= ang && ang < 5 * M_PI / 4) return 3;
    return 2;
}

/* np.angle of n complex values (re, im interleaved), as the model above */
void oracle_np_angle(const double *d, int64_t n, double *ang)
{
    for (int64_t k = 0; k < n; ++k) ang[k] = np_angle(d[2 * k], d[2 * k + 1]);
}

/* The slicer alone over n differential products (re, im interleaved):
 * dibits[k] = 2*hi + lo (tests/test_oracle_slicer.py). */
void oracle_qpsk_slice(const double *d, int64_t n, uint8_t *dibits)
{
    for (int64_t k = 0; k < n; ++k) dibits[k] = (uint8_t)qpsk_dibit(d[2 * k], d[2 * k + 1]);
}

/* ---- sync + pack (modem.py:244-264) -------------------------------------- */
static const uint8_t SYNC16[16] = {0,1,0,0,0,1,1,0, 0,1,0,0,0,0,1,0};   /* "FB" */

int64_t oracle_find_sync(const uint8_t *bits, int64_t L)
{
    for (int64_t p = 0; p + 16 <= L; ++p) {
        int k = 0;
        while (k < 16 && bits[p + k] == SYNC16[k]) ++k;
        if (k == 16) return p;
    }
    return -1;
}

int64_t oracle_pack(const uint8_t *bits, int64_t L, int64_t start, uint8_t *out)
{
    int64_t nb = (L - start) / 8;
    if (nb < 0) nb = 0;
    for (int64_t j = 0; j < nb; ++j) {
        uint8_t v = 0;
        for (int k = 0; k < 8; ++k) v = (uint8_t)((v << 1) | bits[start + 8 * j + k]);
        out[j] = v;
    }
    return nb;
}

/* ---- DPSK demod (QPSK modem.py:189-266, BPSK modem.py:68-135) ---------------
 * kind 0 = DQPSK slicer, 1 = DBPSK slicer.  first = index of the first symbol
 * sample (QPSK sps/2, BPSK sps).  lo: 2*n doubles (re, im interleaved).
 * out must hold (2*n/sps)/8 + 1 bytes.  Returns the byte count, or
 * -1 (n <= BP padlen) / -2 (n <= LP padlen).  *sync_out = sync index or -1. */
int64_t oracle_psk_demod(int kind, const void *x, int dtype, int64_t n,
                         int64_t sps, int64_t first,
                         const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                         const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                         const double *lo, uint8_t *out, int64_t *sync_out)
{
    *sync_out = -1;
    int64_t m = n + 2 * 3 * (int64_t)(bp_nt > lp_nt ? bp_nt : lp_nt);
    double *filt = (double *)malloc(sizeof(double) * n);
    double *re = (double *)malloc(sizeof(double) * n);
    double *im = (double *)malloc(sizeof(double) * n);
    double *work = (double *)malloc(sizeof(double) * 2 * m);
    int64_t result = 0;
    uint8_t *bits = NULL;
    if (oracle_filtfilt(bp_b, bp_a, bp_nt, bp_zi, x, dtype, n, filt, work)) { result = -1; goto done; }
    for (int64_t i = 0; i < n; ++i)                  /* modem.py:200-201: (f + 0j) * lo */
        cmul_np(filt[i], 0.0, lo[2 * i], lo[2 * i + 1], &re[i], &im[i]);
    if (filtfilt_complex(lp_b, lp_a, lp_nt, lp_zi, re, im, n, work)) { result = -2; goto done; }
    {
        int64_t S = (n > first) ? (n - first + sps - 1) / sps : 0;
        if (S < 2) { result = 0; goto done; }        /* modem.py:95-96, 211 */
        int bps = (kind == 0) ? 2 : 1;
        int64_t L = (S - 1) * bps;
        bits = (uint8_t *)malloc((size_t)L + 16);
        for (int64_t k = 0; k + 1 < S; ++k) {
            const double ar = re[first + (k + 1) * sps], ai = im[first + (k + 1) * sps];
            const double br = re[first + k * sps], bi = -im[first + k * sps];   /* conj */
            double dr, di;
            cmul_np(ar, ai, br, bi, &dr, &di);
            if (kind == 1) {
                bits[k] = (dr < 0) ? 1 : 0;              /* modem.py:103-105 */
                continue;
            }
            const int db = qpsk_dibit(dr, di);           /* modem.py:219-241 */
            bits[2 * k] = (uint8_t)(db >> 1);
            bits[2 * k + 1] = (uint8_t)(db & 1);
        }
        int64_t s = oracle_find_sync(bits, L);
        *sync_out = s;
        result = oracle_pack(bits, L, s < 0 ? 0 : s, out);
    }
done:
    free(filt); free(re); free(im); free(work); free(bits);
    return result;
}

/* ---- the time-split layout, restated (psk_split_kernels.hip) -----------------
 * NOT a reference function: the GPU's chunk-parallel approximation of the
 * four filtfilt passes, so tests can check the device computes exactly what
 * DESIGN.md §3.3 says (symbols equal to these up to the sign of a zero) and
 * measure its error against the serial (reference) symbols.  Every pass is cut
 * into chunks of L outputs; a chunk runs the recursion from w samples before
 * its first output from a zero state, or from the pass's start with scipy's
 * zi * first-sample state when that is within w.  The low-pass runs its two
 * components as separate real recursions (the GPU's form; scipy's complex
 * lfilter differs only in signed zeros).  sym: [S][2]. Returns S (0: < 2). */
/* warm_fma: a chunk's steps before its first output (the warm-up) in the
 * GPU's FMA form (psk_common.h bp_warm): y = fma(b0, x, z0),
 * z[i] = fma(-a[i+1], y, fma(b[i+1], x, z[i+1])), z[last] = fma(-a[nt-1], y, b[nt-1] x). */
static void chunked_pass_w(const double *b, const double *a, int nt, const double *zi,
                           const double *in, double *out, int64_t m, int64_t L, int64_t w, int warm_fma)
{
    double z[32];
    for (int64_t o0 = 0; o0 < m; o0 += L) {
        const int64_t o1 = o0 + L < m ? o0 + L : m;
        int64_t j = o0 - w;
        if (j <= 0) { j = 0; for (int i = 0; i < nt - 1; ++i) z[i] = zi[i] * in[0]; }
        else for (int i = 0; i < nt - 1; ++i) z[i] = 0.0;
        for (; j < o1; ++j) {
            if (warm_fma && j < o0) {
                const double x = in[j], y = fma(b[0], x, z[0]);
                for (int i = 0; i < nt - 2; ++i) z[i] = fma(-a[i + 1], y, fma(b[i + 1], x, z[i + 1]));
                z[nt - 2] = fma(-a[nt - 1], y, b[nt - 1] * x);
                continue;
            }
            double y;
            df2t(b, a, nt, z, in + j, &y, 1, 1);
            if (j >= o0) out[j] = y;
        }
    }
}
/* conv_state: psk_split_kernels.hip KS0 restated -- a chunk's start state as
 * Z0[o0] in[0] + sum_{m < min(o0, w)} K[m] in[o0 - 1 - m] (the Z0 term while
 * o0 <= w; zi * in[0] for o0 = 0), summed as the wave does: 64 partial sums,
 * lane l over m = l (mod 64) ascending with fma, then the butterfly
 * p[l] + p[l ^ d] for d = 1, 2, ..., 32, lane 0's value.  K [w][ns], Z0
 * [w + 1][ns] (amr_split_state_tables). */
static void conv_state(const double *K, const double *Z0, int ns, const double *in, int64_t o0, int64_t w,
                       double *z)
{
    double p[64][16], q[64][16];
    if (o0 == 0) { for (int i = 0; i < ns; ++i) z[i] = Z0[i] * in[0]; return; }
    for (int l = 0; l < 64; ++l) for (int i = 0; i < ns; ++i) p[l][i] = 0.0;
    const int64_t M = o0 < w ? o0 : w;
    for (int64_t m = 0; m < M; ++m)
        for (int i = 0; i < ns; ++i) p[m & 63][i] = fma(K[m * ns + i], in[o0 - 1 - m], p[m & 63][i]);
    for (int d = 1; d < 64; d <<= 1) {
        for (int l = 0; l < 64; ++l) for (int i = 0; i < ns; ++i) q[l][i] = p[l][i] + p[l ^ d][i];
        memcpy(p, q, sizeof(p));
    }
    for (int i = 0; i < ns; ++i) z[i] = o0 <= w ? fma(Z0[o0 * ns + i], in[0], p[0][i]) : p[0][i];
}
/* a chunked pass whose chunks start from conv_state (no warm-up steps) */
static void chunked_pass_conv(const double *b, const double *a, int nt, const double *in, double *out, int64_t m,
                              int64_t L, int64_t w, const double *K, const double *Z0)
{
    double z[32];
    for (int64_t o0 = 0; o0 < m; o0 += L) {
        const int64_t o1 = o0 + L < m ? o0 + L : m;
        conv_state(K, Z0, nt - 1, in, o0, w, z);
        for (int64_t j = o0; j < o1; ++j) df2t(b, a, nt, z, in + j, &out[j], 1, 1);
    }
}
/* The strict mode's statistics of one convolution-started chunked pass
 * (psk_split_kernels.hip KS0 + KS1 / KS2 with PskSplit::strict, restated):
 * per chunk c the start-state bound ds[c] = gam (sum_m kabs[m] |in[o0-1-m]|
 * + z0abs[o0] |in[0]|) (0 for c = 0) summed as the wave does (lane l over m =
 * l mod 64 with fma, then the butterfly); per output step the rounding bound
 * fma(u2, sz, fma(kx, |x|, ky |y|)), sz the pre-step |z1..z7| in the
 * kernel's pairing, summed per block of 16 outputs in step order (dblk) and
 * maximised (*dmax); *ymax: max |out| over [olo, ohi).  cst: u2, kx, ky, gam.
 * L must be a multiple of 16. */
static void chunked_pass_conv_stats(const double *b, const double *a, int nt, const double *in, double *out,
                                    int64_t m, int64_t L, int64_t w, const double *K, const double *Z0,
                                    const double *kabs, const double *z0abs, const double *cst, int64_t olo,
                                    int64_t ohi, double *dblk, double *ds, double *dmax, double *ymax)
{
    double z[32];
    for (int64_t o0 = 0, c = 0; o0 < m; o0 += L, ++c) {
        const int64_t o1 = o0 + L < m ? o0 + L : m;
        conv_state(K, Z0, nt - 1, in, o0, w, z);
        ds[c] = 0.0;
        if (o0 > 0) {
            double p[64], q[64];
            for (int l = 0; l < 64; ++l) p[l] = 0.0;
            const int64_t M = o0 < w ? o0 : w;
            for (int64_t mm = 0; mm < M; ++mm) p[mm & 63] = fma(kabs[mm], fabs(in[o0 - 1 - mm]), p[mm & 63]);
            for (int d = 1; d < 64; d <<= 1) {
                for (int l = 0; l < 64; ++l) q[l] = p[l] + p[l ^ d];
                memcpy(p, q, sizeof(p));
            }
            const double z0t = o0 <= w ? z0abs[o0] * fabs(in[0]) : 0.0;
            ds[c] = cst[3] * (p[0] + z0t);
        }
        double dsum = 0.0;
        int cnt = 0;
        for (int64_t j = o0; j < o1; ++j) {
            /* the kernels' pairing: 8 states (psk_split_kernels.hip step_bound_pre),
             * 6 states (fsk_kernels.hip fsk_step_sz) */
            const double sz = nt == 9 ? ((fabs(z[1]) + fabs(z[2])) + (fabs(z[3]) + fabs(z[4]))) +
                                            ((fabs(z[5]) + fabs(z[6])) + fabs(z[7]))
                                      : ((fabs(z[1]) + fabs(z[2])) + (fabs(z[3]) + fabs(z[4]))) + fabs(z[5]);
            df2t(b, a, nt, z, in + j, &out[j], 1, 1);
            const double dd = fma(cst[0], sz, fma(cst[1], fabs(in[j]), cst[2] * fabs(out[j])));
            if (dd > *dmax) *dmax = dd;
            dsum += dd;
            if (++cnt == 16) { dblk[j / 16] = dsum; dsum = 0.0; cnt = 0; }
            if (j >= olo && j < ohi && fabs(out[j]) > *ymax) *ymax = fabs(out[j]);
        }
        if (cnt > 0) dblk[(o1 - 1) / 16] = dsum;
    }
}

static void chunked_pass(const double *b, const double *a, int nt, const double *zi,
                         const double *in, double *out, int64_t m, int64_t L, int64_t w)
{
    chunked_pass_w(b, a, nt, zi, in, out, m, L, w, 0);
}

/* The FSK time-split F1 (fsk_kernels.hip FS1 / FS2), restated per tone: the
 * chunked forward pass over the odd-extended input, the chunked backward pass
 * over its reversal, f[i] = y[m - 1 - pad - i].  Same chunk rule as
 * chunked_pass (zero start w samples early, scipy's zi state for the chunk
 * at the pass's start, warm-up steps in FMA form).  out: n doubles.
 * Returns -1 if n <= pad. */
int oracle_split_filtfilt(const double *b, const double *a, int nt, const double *zi, const void *x, int dtype,
                          int64_t n, int64_t L, int64_t w, const double *K, const double *Z0, double *out)
{
    /* K, Z0 (both or neither): chunks start from conv_state (FS0, the GPU's
     * default), else from w-step FMA-form warm-ups */
    const int pad = 3 * nt;
    if (n <= pad || L < 1) return -1;
    const int64_t m = n + 2 * (int64_t)pad;
    double *e = (double *)malloc(sizeof(double) * (size_t)m);
    double *y = (double *)malloc(sizeof(double) * (size_t)m);
    double *r = (double *)malloc(sizeof(double) * (size_t)m);
    for (int64_t j = 0; j < m; ++j) e[j] = ext_sample(x, dtype, n, pad, j);
    if (K && Z0 && nt <= 17) {
        chunked_pass_conv(b, a, nt, e, y, m, L, w, K, Z0);
        for (int64_t k = 0; k < m; ++k) r[k] = y[m - 1 - k];
        chunked_pass_conv(b, a, nt, r, y, m, L, w, K, Z0);
    } else {
        chunked_pass_w(b, a, nt, zi, e, y, m, L, w, 1);
        for (int64_t k = 0; k < m; ++k) r[k] = y[m - 1 - k];
        chunked_pass_w(b, a, nt, zi, r, y, m, L, w, 1);
    }
    for (int64_t i = 0; i < n; ++i) out[i] = y[m - 1 - pad - i];
    free(e); free(y); free(r);
    return 0;
}

int64_t oracle_psk_split_symbols(const void *x, int dtype, int64_t n, int64_t sps, int64_t first,
                                 const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                                 const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                                 const double *lo, int64_t L, int64_t w1, int64_t w2, const double *K,
                                 const double *Z0, double *sym)
{
    /* K, Z0 (both or neither): the band-pass chunks start from conv_state
     * (the GPU's default), else from w1-step FMA-form warm-ups */
    const int pad1 = 3 * bp_nt, pad2 = 3 * lp_nt;
    if (n <= pad1 || n <= pad2 || L < 1) return -1;
    const int64_t S = (n > first) ? (n - first + sps - 1) / sps : 0;
    if (S < 2) return 0;
    const int64_t m1 = n + 2 * (int64_t)pad1, m2 = n + 2 * (int64_t)pad2;
    double *e = (double *)malloc(sizeof(double) * (size_t)(m1 > 2 * m2 ? m1 : 2 * m2));
    double *y = (double *)malloc(sizeof(double) * (size_t)m1);
    double *r = (double *)malloc(sizeof(double) * (size_t)m1);
    double *g = (double *)malloc(sizeof(double) * 2 * (size_t)n);
    for (int64_t j = 0; j < m1; ++j) e[j] = ext_sample(x, dtype, n, pad1, j);
    if (K && Z0 && bp_nt <= 17) {
        chunked_pass_conv(bp_b, bp_a, bp_nt, e, y, m1, L, w1, K, Z0);
        for (int64_t k = 0; k < m1; ++k) r[k] = y[m1 - 1 - k];
        chunked_pass_conv(bp_b, bp_a, bp_nt, r, y, m1, L, w1, K, Z0);
    } else {
        chunked_pass_w(bp_b, bp_a, bp_nt, bp_zi, e, y, m1, L, w1, 1);
        for (int64_t k = 0; k < m1; ++k) r[k] = y[m1 - 1 - k];
        chunked_pass_w(bp_b, bp_a, bp_nt, bp_zi, r, y, m1, L, w1, 1);
    }
    for (int64_t i = 0; i < n; ++i)                      /* f[i] = y[m1 - 1 - pad1 - i]; (f + 0j) * lo */
        cmul_np(y[m1 - 1 - pad1 - i], 0.0, lo[2 * i], lo[2 * i + 1], &g[2 * i], &g[2 * i + 1]);
    for (int c = 0; c < 2; ++c) {
        double *ec = e + (size_t)c * m2;
        const double x0 = g[c], xl = g[2 * (n - 1) + c];
        for (int j = 0; j < pad2; ++j) ec[j] = 2.0 * x0 - g[2 * (pad2 - j) + c];
        for (int64_t i = 0; i < n; ++i) ec[pad2 + i] = g[2 * i + c];
        for (int j = 0; j < pad2; ++j) ec[pad2 + n + j] = 2.0 * xl - g[2 * (n - 2 - j) + c];
        chunked_pass(lp_b, lp_a, lp_nt, lp_zi, ec, y, m2, L, w2);
        for (int64_t k = 0; k < m2; ++k) r[k] = y[m2 - 1 - k];
        chunked_pass(lp_b, lp_a, lp_nt, lp_zi, r, y, m2, L, w2);
        for (int64_t q = 0; q < S; ++q) sym[2 * q + c] = y[m2 - 1 - pad2 - (first + q * sps)];
    }
    free(e); free(y); free(r); free(g);
    return S;
}

/* The strict mode's per-stream statistics of the split band-pass passes
 * (restating the device's; tests compute the bound from them): d1, d2 [nb1]
 * the passes' per-block step bound sums (nb1 = ceil(m1 / 16)), ds1, ds2 [c1]
 * their chunk-start bounds (c1 = ceil(m1 / L)), stats[4] = D1max, max|y1|,
 * D2max, max|f|.  Returns 0, or -1 for bad arguments (bp_nt 9: the PSK
 * kernels' 8 states, or 7: the FSK split F1's 6 (fsk_kernels.hip FS0-FS2 with
 * the strict step bounds, one tone); L a multiple of 16). */
int oracle_psk_split_stats(const void *x, int dtype, int64_t n, const double *bp_b, const double *bp_a, int bp_nt,
                           int64_t L, int64_t w1, const double *K, const double *Z0, const double *kabs,
                           const double *z0abs, const double *cst, double *d1, double *d2, double *ds1, double *ds2,
                           double *stats)
{
    const int pad1 = 3 * bp_nt;
    if ((bp_nt != 9 && bp_nt != 7) || n <= pad1 || L < 16 || L % 16 || !K || !Z0) return -1;
    const int64_t m1 = n + 2 * (int64_t)pad1;
    double *e = (double *)malloc(sizeof(double) * (size_t)m1);
    double *y = (double *)malloc(sizeof(double) * (size_t)m1);
    double *r = (double *)malloc(sizeof(double) * (size_t)m1);
    for (int i = 0; i < 4; ++i) stats[i] = 0.0;
    for (int64_t j = 0; j < m1; ++j) e[j] = ext_sample(x, dtype, n, pad1, j);
    chunked_pass_conv_stats(bp_b, bp_a, bp_nt, e, y, m1, L, w1, K, Z0, kabs, z0abs, cst, 0, m1, d1, ds1, &stats[0],
                            &stats[1]);
    for (int64_t k = 0; k < m1; ++k) r[k] = y[m1 - 1 - k];
    /* f[i] = y[m1 - 1 - pad1 - i], i in [0, n) <-> pass-2 index k in [pad1, pad1 + n) */
    chunked_pass_conv_stats(bp_b, bp_a, bp_nt, r, y, m1, L, w1, K, Z0, kabs, z0abs, cst, pad1, pad1 + n, d2, ds2,
                            &stats[2], &stats[3]);
    free(e); free(y); free(r);
    return 0;
}

/* The serial (reference) symbol samples baseband[first::sps] of the same
 * stream: scipy's filtfilt, the mixer, scipy's complex filtfilt.  sym [S][2].
 * f32f: the band-pass output rounded to float32 before the mixer -- NOT the
 * reference: the lane layout's float32 hand-off, restated. */
static int64_t psk_symbols(const void *x, int dtype, int64_t n, int64_t sps, int64_t first,
                           const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                           const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                           const double *lo, double *sym, int f32f);
int64_t oracle_psk_symbols(const void *x, int dtype, int64_t n, int64_t sps, int64_t first,
                           const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                           const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                           const double *lo, double *sym)
{
    return psk_symbols(x, dtype, n, sps, first, bp_b, bp_a, bp_nt, bp_zi, lp_b, lp_a, lp_nt, lp_zi, lo, sym, 0);
}
int64_t oracle_psk_symbols_f32f(const void *x, int dtype, int64_t n, int64_t sps, int64_t first,
                                const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                                const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                                const double *lo, double *sym, double *fpeak)
{
    /* fpeak: max |f| (the kernel's per-stream scale of the margin) */
    int64_t m = n + 2 * 3 * (int64_t)(bp_nt > lp_nt ? bp_nt : lp_nt);
    double *filt = (double *)malloc(sizeof(double) * n);
    double *work = (double *)malloc(sizeof(double) * 2 * m);
    *fpeak = 0.0;
    if (oracle_filtfilt(bp_b, bp_a, bp_nt, bp_zi, x, dtype, n, filt, work) == 0)
        for (int64_t i = 0; i < n; ++i) if (fabs(filt[i]) > *fpeak) *fpeak = fabs(filt[i]);
    free(filt); free(work);
    return psk_symbols(x, dtype, n, sps, first, bp_b, bp_a, bp_nt, bp_zi, lp_b, lp_a, lp_nt, lp_zi, lo, sym, 1);
}
static int64_t psk_symbols(const void *x, int dtype, int64_t n, int64_t sps, int64_t first,
                           const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                           const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                           const double *lo, double *sym, int f32f)
{
    const int64_t S = (n > first) ? (n - first + sps - 1) / sps : 0;
    int64_t m = n + 2 * 3 * (int64_t)(bp_nt > lp_nt ? bp_nt : lp_nt);
    double *filt = (double *)malloc(sizeof(double) * n);
    double *re = (double *)malloc(sizeof(double) * n);
    double *im = (double *)malloc(sizeof(double) * n);
    double *work = (double *)malloc(sizeof(double) * 2 * m);
    int64_t rc = S;
    if (oracle_filtfilt(bp_b, bp_a, bp_nt, bp_zi, x, dtype, n, filt, work)) rc = -1;
    else {
        if (f32f) for (int64_t i = 0; i < n; ++i) filt[i] = (double)(float)filt[i];
        for (int64_t i = 0; i < n; ++i) cmul_np(filt[i], 0.0, lo[2 * i], lo[2 * i + 1], &re[i], &im[i]);
        if (filtfilt_complex(lp_b, lp_a, lp_nt, lp_zi, re, im, n, work)) rc = -2;
        else for (int64_t q = 0; q < S; ++q) { sym[2 * q] = re[first + q * sps]; sym[2 * q + 1] = im[first + q * sps]; }
    }
    free(filt); free(re); free(im); free(work);
    return rc;
}

/* Batch driver (the CPU baseline): streams are independent; parallelised with
 * OpenMP across streams when built with -fopenmp. */
int64_t oracle_psk_demod_batch(int kind, const void *x, int dtype, int64_t n_streams, int64_t n,
                               int64_t x_stride, int64_t sps, int64_t first,
                               const double *bp_b, const double *bp_a, int bp_nt, const double *bp_zi,
                               const double *lp_b, const double *lp_a, int lp_nt, const double *lp_zi,
                               const double *lo, uint8_t *out, int64_t out_stride,
                               int64_t *out_len, int64_t *sync_idx, int n_threads)
{
    const size_t esz = dt_size(dtype);
    int64_t worst = 0;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(n_threads) reduction(min:worst)
#endif
    for (int64_t s = 0; s < n_streams; ++s) {
        const void *xs = (const char *)x + (size_t)s * (size_t)x_stride * esz;
        int64_t r = oracle_psk_demod(kind, xs, dtype, n, sps, first, bp_b, bp_a, bp_nt, bp_zi,
                                     lp_b, lp_a, lp_nt, lp_zi, lo, out + s * out_stride, &sync_idx[s]);
        out_len[s] = r;
        if (r < worst) worst = r;
    }
    (void)n_threads;
    return worst;
}

/* ---- FSK decision stage (modem.py:315-341) ----------------------------------
 * Given the two envelopes, reproduce the per-sample compare, the windowed
 * majority vote and sync+pack.  Returns the byte count. */
int64_t oracle_fsk_decide(const double *mark_env, const double *space_env, int64_t n,
                          int64_t sps, uint8_t *out, int64_t *sync_out)
{
    int64_t half = sps / 2, q = sps / 4;
    int64_t nb = 0;
    uint8_t *dec = (uint8_t *)malloc((size_t)(n / (sps > 0 ? sps : 1) + 2));
    for (int64_t i = half; i < n; i += sps) {
        int64_t lo = i - q, hi = i + q < n ? i + q : n;
        if (hi - lo <= 0) continue;                      /* len(chunk) > 0 */
        int64_t ones = 0;
        for (int64_t j = lo; j < hi; ++j) ones += mark_env[j] > space_env[j];
        dec[nb++] = (2 * ones > hi - lo) ? 1 : 0;        /* np.mean(chunk) > 0.5 */
    }
    int64_t s = oracle_find_sync(dec, nb);
    *sync_out = s;
    int64_t r = oracle_pack(dec, nb, s < 0 ? 0 : s, out);
    free(dec);
    return r;
}

/* ---- FEC (fec.py:11-69) ------------------------------------------------------ */
uint32_t oracle_crc32(const uint8_t *p, int64_t n)
{
    uint32_t c = 0xFFFFFFFFu;
    for (int64_t i = 0; i < n; ++i) {
        c ^= p[i];
        for (int k = 0; k < 8; ++k) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
    }
    return c ^ 0xFFFFFFFFu;
}

/* Returns decoded length; *crc_ok = 1 when the recomputed CRC32 matches the
 * trailing little-endian word (the reference only prints on mismatch). */
int64_t oracle_fec_decode(const uint8_t *in, int64_t n, uint8_t *out, int *crc_ok)
{
    if (n < 4) {                                   /* fec.py:36-37: returned as is */
        memcpy(out, in, (size_t)n);
        *crc_ok = 1;
        return n;
    }
    const uint32_t want = (uint32_t)in[n - 4] | ((uint32_t)in[n - 3] << 8) |
                          ((uint32_t)in[n - 2] << 16) | ((uint32_t)in[n - 1] << 24);
    const int64_t m = n - 4;
    int64_t o = 0, i = 0;
    while (i < m) {
        if (i + 2 < m) {
            const uint8_t b1 = in[i], b2 = in[i + 1], p = in[i + 2];
            out[o++] = b1;
            out[o++] = ((b1 ^ b2) == p) ? b2 : 0x3F;
            i += 3;
        } else {
            out[o++] = in[i++];
        }
    }
    *crc_ok = oracle_crc32(out, o) == want;
    return o;
}
