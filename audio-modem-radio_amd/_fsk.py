"""FSK host layer: filter design with the reference's scipy calls + GPU launch.

fsk_demodulate (modem.py:298-341): per tone butter(3, [(f-baud)/nyq, (f+baud)/nyq],
'band') WITHOUT clamping -- scipy raises for an edge <= 0 or >= 1, which is the
reference's behaviour at its own defaults -- then filtfilt,
|hilbert|, per-sample compare, windowed majority, sync + pack.  Everything
after the filter design runs in libamr.so (fsk_kernels.hip, fft_kernels.hip).
"""
from __future__ import annotations

import ctypes
import functools
import threading

import numpy as np

import _amr
from _amr import check, lib, ptr


def design_fsk(n: int, baud, mark_freq, space_freq, samp_rate):
    """Return (sps, [(b, a, zi) mark, (b, a, zi) space]); raise exactly where
    the reference raises, in the reference's order (modem.py:301-320).
    Memoised per parameter set (scipy's butter + lfilter_zi for both tones
    took ~0.3-0.6 ms of every one-capture call); the arrays are read-only,
    and a raising design is not cached (it raises again on every call)."""
    return _design_fsk(int(n), baud, mark_freq, space_freq, samp_rate)


@functools.lru_cache(maxsize=256)
def _design_fsk(n: int, baud, mark_freq, space_freq, samp_rate):
    from scipy import signal
    sps = int(samp_rate / baud)            # modem.py:301 (ZeroDivisionError for baud == 0)
    nyq = samp_rate / 2
    out = []
    for f in (mark_freq, space_freq):      # mark envelope is computed first (modem.py:311-312)
        b, a = signal.butter(3, [(f - baud) / nyq, (f + baud) / nyq], btype='band')
        nt = max(len(a), len(b))
        if n <= 3 * nt:
            raise ValueError("The length of the input vector x must be greater than padlen, which is %d." % (3 * nt))
        arrs = tuple(np.ascontiguousarray(v, np.float64) for v in (b, a, signal.lfilter_zi(b, a)))
        for v in arrs:
            v.setflags(write=False)
        out.append(arrs)
    if sps == 0:
        raise ValueError("range() arg 3 must not be zero")   # modem.py:320
    return sps, out


FSK_LAYOUTS = {"auto": 0, "serial": 1, "split": 2}


def split_design(n: int, baud, mark_freq, space_freq, samp_rate=96000):
    """The FSK time-split design (host arithmetic in libamr.so, no device):
    dict of warmup, kappa, hilbert_l1, tau (F2's margin scale for split calls),
    or None when the filters cannot be split at this length."""
    _, ((mb, ma, _), (sb, sa, _)) = design_fsk(n, baud, mark_freq, space_freq, samp_rate)
    w, k, h = ctypes.c_int64(0), ctypes.c_double(0.0), ctypes.c_double(0.0)
    rc = lib().amr_fsk_split_design(int(n), ptr(mb), ptr(ma), ptr(sb), ptr(sa), len(mb), ctypes.byref(w),
                                    ctypes.byref(k), ctypes.byref(h))
    if rc != 0:
        return None
    m = fft_margin(n, baud, mark_freq, space_freq, samp_rate)
    return {"warmup": w.value, "kappa": k.value, "hilbert_l1": h.value, "tau": m["tau"] + k.value * h.value}


def split_strict_design(n: int, baud, mark_freq, space_freq, samp_rate=96000):
    """The split F1's strict band-pass design per tone (libamr.so host
    arithmetic, amr_fsk_split_strict_design): [mark, space] dicts of the
    constants (_amr.STRICT_CONSTS) and the tables kabs, z0abs, W, K12, HS, GS,
    TZ; None when there is no split design or no strict bound."""
    sd = split_design(n, baud, mark_freq, space_freq, samp_rate)
    if sd is None:
        return None
    _, tones = design_fsk(n, baud, mark_freq, space_freq, samp_rate)
    out = []
    for b, a, zi in tones:
        c = np.zeros(32)
        if lib().amr_fsk_split_strict_design(ptr(b), ptr(a), ptr(zi), len(b), int(sd["warmup"]), ptr(c), None) != 0:
            return None
        d = dict(zip(_amr.STRICT_CONSTS, c[:len(_amr.STRICT_CONSTS)].tolist()))
        w = int(d["w1"])
        sizes = [("kabs", w), ("z0abs", w + 1), ("W", int(d["nw"])), ("K12", int(d["nk"])), ("HS", int(d["nh"])),
                 ("GS", int(d["ng"])), ("TZ", int(d["nz"]))]
        tabs = np.zeros(sum(k for _, k in sizes))
        check(lib().amr_fsk_split_strict_design(ptr(b), ptr(a), ptr(zi), len(b), w, ptr(c), ptr(tabs)))
        o = 0
        for name, k in sizes:
            d[name] = tabs[o:o + k]
            o += k
        out.append(d)
    return out


def fft_margin(n: int, baud, mark_freq, space_freq, samp_rate=96000):
    """F2's margin scale from a standard FFT rounding bound (host arithmetic
    in libamr.so, no device; include/amr.h amr_fsk_fft_margin): dict of tau,
    eps_fast, eps_ref, zmax (the bound on max_t ||z_t||_2 / peak|ext x|),
    fast_blue, fast_M, ref_blue, ref_M."""
    _, ((mb, ma, mz), (sb, sa, sz)) = design_fsk(n, baud, mark_freq, space_freq, samp_rate)
    out = np.zeros(8)
    check(lib().amr_fsk_fft_margin(int(n), ptr(mb), ptr(ma), ptr(mz), ptr(sb), ptr(sa), ptr(sz), len(mb), ptr(out)))
    return {"tau": out[0], "eps_fast": out[1], "eps_ref": out[2], "zmax": out[3], "fast_blue": bool(out[4]),
            "fast_M": int(out[5]), "ref_blue": bool(out[6]), "ref_M": int(out[7])}


class FskPlan:
    """A device plan: both tones' coefficients, the FFT tables and HBM scratch."""

    def __init__(self, n: int, baud, mark_freq, space_freq, samp_rate=96000, max_streams=64, device=None):
        self.n = int(n)
        self.sps, ((mb, ma, mzi), (sb, sa, szi)) = design_fsk(n, baud, mark_freq, space_freq, samp_rate)
        self.coef = (mb, ma, mzi, sb, sa, szi)
        _amr.require_gpu()
        self.device = _amr.default_device() if device is None else device
        self.max_streams = int(max_streams)
        self.handle = None
        self.out_cap = 1
        self.lock = threading.Lock()
        if self.sps < 0:
            return      # range(sps//2, n, sps) with a negative step is empty: b'' for every stream
        h = ctypes.c_void_p()
        check(lib().amr_fsk_plan_create(ctypes.byref(h), self.device, self.n, self.sps, ptr(mb), ptr(ma), ptr(mzi),
                                        ptr(sb), ptr(sa), ptr(szi), len(mb), self.max_streams))
        self.handle = h
        self.out_cap = int(lib().amr_fsk_plan_out_capacity(h))
        self.fft_length = int(lib().amr_fsk_plan_fft_length(h))
        self.live_columns = bool(lib().amr_fsk_plan_live_columns(h))

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _amr._lib is not None:
            try:
                _amr._lib.amr_fsk_plan_destroy(h)
            except Exception:
                pass
            self.handle = None

    def _chunks(self, x):
        x = np.ascontiguousarray(x)
        if x.dtype not in _amr.DTYPES:
            x = np.ascontiguousarray(x, np.float64)
        for s0 in range(0, x.shape[0], self.max_streams):
            yield s0, x[s0:s0 + self.max_streams]

    def demod_host(self, x: np.ndarray):
        """x [B][N] float32/float64/int16. Returns (list[bytes], sync[B])."""
        B = x.shape[0]
        if self.handle is None:
            return [b""] * B, np.full(B, -1, np.int64)
        outs, syncs = [], np.empty(B, np.int64)
        cap = max(self.out_cap, 1)
        for s0, xb in self._chunks(x):
            nb = xb.shape[0]
            out = np.empty((nb, cap), np.uint8)
            ln = np.empty(nb, np.int64)
            sy = np.empty(nb, np.int64)
            with self.lock:
                check(lib().amr_fsk_demod_host(self.handle, ptr(xb), _amr.DTYPES[xb.dtype], nb, xb.shape[1],
                                               ptr(out), cap, ptr(ln), ptr(sy)))
            outs += [out[i, :ln[i]].tobytes() for i in range(nb)]
            syncs[s0:s0 + nb] = sy
        return outs, syncs

    def demod_host_raw(self, x: np.ndarray):
        """x [B][N] of a dtype the kernels do not store (_amr.raw_input): the
        reference's semantics for that array (both tones' filtfilt see the
        same odd extension).  Returns (list[bytes], sync[B])."""
        B = x.shape[0]
        if self.handle is None:
            return [b""] * B, np.full(B, -1, np.int64)
        xk, edges = _amr.raw_input(x, 3 * len(self.coef[0]))
        outs, syncs = [], np.empty(B, np.int64)
        cap = max(self.out_cap, 1)
        for s0 in range(0, B, self.max_streams):
            xb, eb = xk[s0:s0 + self.max_streams], edges[s0:s0 + self.max_streams]
            nb = xb.shape[0]
            out = np.empty((nb, cap), np.uint8)
            ln = np.empty(nb, np.int64)
            sy = np.empty(nb, np.int64)
            with self.lock:
                check(lib().amr_fsk_demod_host_edges(self.handle, ptr(xb), _amr.DTYPES[xb.dtype], nb, xb.shape[1],
                                                     ptr(eb), ptr(out), cap, ptr(ln), ptr(sy)))
            outs += [out[i, :ln[i]].tobytes() for i in range(nb)]
            syncs[s0:s0 + nb] = sy
        return outs, syncs

    def envelopes(self, x: np.ndarray):
        """(mark_env, space_env) [B][N]: |hilbert(filtfilt(.))| per tone (modem.py:308-309)."""
        if self.handle is None:
            raise _amr.AmrError(_amr.AMR_E_INVALID, "plan has no decision path (sps < 0)")
        B = x.shape[0]
        m = np.empty((B, self.n))
        s = np.empty((B, self.n))
        for s0, xb in self._chunks(x):
            nb = xb.shape[0]
            with self.lock:
                check(lib().amr_fsk_envelopes_host(self.handle, ptr(xb), _amr.DTYPES[xb.dtype], nb, xb.shape[1],
                                                   ptr(m[s0:s0 + nb]), ptr(s[s0:s0 + nb])))
        return m, s

    def scratch_bytes(self) -> int:
        """Device bytes this plan holds (scratch + host-API staging)."""
        return int(lib().amr_fsk_plan_scratch_bytes(self.handle)) if self.handle else 0

    def resident_bytes(self) -> int:
        """Device bytes allocated now (a device-entry-only plan holds no host staging)."""
        return int(lib().amr_fsk_plan_resident_bytes(self.handle)) if self.handle else 0

    def enable_timing(self, on=True):
        check(lib().amr_fsk_plan_enable_timing(self.handle, 1 if on else 0))

    def set_layout(self, layout: str):
        """F1 per call: "auto" (split for <= 1024 streams), "serial", "split" (include/amr.h)."""
        check(lib().amr_fsk_plan_set_layout(self.handle, FSK_LAYOUTS[layout]))

    def split_conv(self) -> bool:
        """The time-split F1 starts its chunks from convolution states (FS0)
        rather than warm-ups (AMR_FSK_SPLIT_CONV=0)."""
        return int(lib().amr_fsk_plan_split_conv(self.handle)) == 1

    def split_info(self) -> dict:
        """The last call's F1 layout and the plan's split design."""
        ls, w, L = ctypes.c_int(0), ctypes.c_int64(0), ctypes.c_int64(0)
        k, t = ctypes.c_double(0.0), ctypes.c_double(0.0)
        check(lib().amr_fsk_plan_split_info(self.handle, ctypes.byref(ls), ctypes.byref(w), ctypes.byref(L),
                                            ctypes.byref(k), ctypes.byref(t)))
        return {"last_split": bool(ls.value), "warmup": w.value, "chunk": L.value, "kappa": k.value, "tau": t.value}

    def set_split_strict(self, on):
        """The split F1's strict margin for this plan: True / False, None = the
        process default (AMR_FSK_SPLIT_STRICT)."""
        check(lib().amr_fsk_plan_set_split_strict(self.handle, -1 if on is None else (1 if on else 0)))

    def split_strict(self) -> bool:
        return int(lib().amr_fsk_plan_split_strict(self.handle)) == 1

    def last_strict(self) -> bool:
        return int(lib().amr_fsk_plan_last_strict(self.handle)) == 1

    def split_bounds(self, x: np.ndarray):
        """Diagnostic: the strict split F1 over x [B][n] -> (z [B][n][2] (mark,
        space), per-tone maxima [B][2][8] (D1max, E1max, max|y1|, D2max, S1max,
        -, F, -), peak [B] = max |ext x|)."""
        x = np.ascontiguousarray(np.atleast_2d(x))
        if x.dtype not in _amr.DTYPES:
            x = np.ascontiguousarray(x, np.float64)
        B = x.shape[0]
        z = np.zeros((B, self.n, 2))
        bnd = np.zeros((B, 2, 8))
        pk = np.zeros(B)
        with self.lock:
            check(lib().amr_fsk_split_bounds_host(self.handle, ptr(x), _amr.DTYPES[x.dtype], B, x.shape[1], ptr(z),
                                                  ptr(bnd), ptr(pk)))
        return z, bnd, pk

    def margin(self) -> dict:
        """F2's margin scales of this plan: tau (serial F1) and tau_split."""
        t, ts = ctypes.c_double(0.0), ctypes.c_double(0.0)
        check(lib().amr_fsk_plan_margin(self.handle, ctypes.byref(t), ctypes.byref(ts)))
        return {"tau": t.value, "tau_split": ts.value}

    def split_bandpass(self, x: np.ndarray, chunk: int = 0) -> np.ndarray:
        """The split F1's output [B][n][2] (mark, space): a diagnostic."""
        x = np.ascontiguousarray(x)
        if x.dtype not in _amr.DTYPES:
            x = np.ascontiguousarray(x, np.float64)
        out = np.empty((x.shape[0], self.n, 2))
        with self.lock:
            check(lib().amr_fsk_split_bandpass_host(self.handle, ptr(x), _amr.DTYPES[x.dtype], x.shape[0], x.shape[1],
                                                    int(chunk), ptr(out)))
        return out

    def set_exact_mode(self, mode: int):
        """0 off, 1 the streams F2 flags (default), 2 every stream (include/amr.h)."""
        check(lib().amr_fsk_plan_set_exact_mode(self.handle, int(mode)))

    def exact_streams(self) -> int:
        """Streams the exact path recomputed in the last call (F2 flagged them)."""
        c = ctypes.c_int64(0)
        check(lib().amr_fsk_plan_exact_streams(self.handle, ctypes.byref(c)))
        return int(c.value)

    def timings(self) -> dict:
        ms = (ctypes.c_float * len(_amr.TF_NAMES))()
        check(lib().amr_fsk_plan_timings(self.handle, ms, len(_amr.TF_NAMES)))
        return {k: float(v) for k, v in zip(_amr.TF_NAMES, ms) if v >= 0}


MAX_CHUNK = 16384


def get_fsk_plan(n, baud, mark_freq, space_freq, samp_rate, batch) -> FskPlan:
    """From the drop-in path's one plan cache (_amr.plan_cache, shared with PSK)."""
    dev = _amr.default_device()
    key = ("fsk", int(n), float(baud), float(mark_freq), float(space_freq), float(samp_rate), dev)
    need = max(16, _amr.stream_bucket(batch, MAX_CHUNK))   # the FFT passes tile 8+ rows
    sps = int(samp_rate / baud)

    def estimate(m):
        return max(0, int(lib().amr_fsk_plan_bytes_estimate(int(n), sps, 7, m)))
    return _amr.plan_cache.get(key, need, lambda m: FskPlan(n, baud, mark_freq, space_freq, samp_rate, max_streams=m,
                                                            device=dev), estimate if sps >= 1 else None)


def fsk_demodulate_batch(x: np.ndarray, baud, mark_freq, space_freq, samp_rate, raw=False) -> list:
    """raw: x is the caller's array as the reference gets it (any real dtype;
    int16 as values) -- otherwise the plans' convention (int16 = PCM / 32768,
    decode_wav_file's path)."""
    if x.ndim != 2:
        raise ValueError("batch input must be a 2-D [streams, samples] array")
    design_fsk(x.shape[1], baud, mark_freq, space_freq, samp_rate)
    _amr.require_gpu()
    if x.shape[0] == 0:
        return []
    plan = get_fsk_plan(x.shape[1], baud, mark_freq, space_freq, samp_rate, x.shape[0])
    if raw and not _amr.is_kernel_dtype(x.dtype):
        return plan.demod_host_raw(x)[0]
    return plan.demod_host(x)[0]
