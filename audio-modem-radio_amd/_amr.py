"""ctypes binding of libamr.so (include/amr.h) + the host-side plan cache.

This is the thin host layer between the reference-shaped Python API
(modem.py / decoder.py / fec.py in this directory) and the HIP kernels.
There is deliberately NO CPU fallback: if libamr.so is missing or no GPU is
visible, every demodulation raises AmrError.

Filter design happens here, on the host, with the same scipy calls the
reference makes (modem.py:73-76/86-87 BPSK, modem.py:194-197/203 QPSK), so the
coefficients -- and scipy's ValueError messages -- are the reference's own.
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("AMR_LIB", os.path.join(HERE, "libamr.so"))

AMR_OK = 0
AMR_E_INVALID, AMR_E_PADLEN, AMR_E_HIP, AMR_E_NOMEM, AMR_E_NODEVICE, AMR_E_RCCL, AMR_E_CAPACITY = \
    -1, -2, -3, -4, -5, -6, -7
DTYPE_F32, DTYPE_F64, DTYPE_I16 = 0, 1, 2
PSK_QPSK, PSK_BPSK = 0, 1
T_NAMES = ["bandpass", "lowpass_fwd", "lowpass_bwd", "lowpass_exact", "sync_pack", "fec", "launch"]
TF_NAMES = ["bandpass", "hilbert", "decide", "launch", "exact"]
# amr_frame_rec (include/amr.h), 64 bytes
FRAME_SHORT, FRAME_NONAME, FRAME_NOMETA, FRAME_BADLEN, FRAME_INCOMPLETE, FRAME_CRC_BAD, FRAME_OK = range(7)
FRAME_REC = np.dtype([("start", "<i8"), ("name_start", "<i8"), ("payload_start", "<i8"), ("status", "<i4"),
                      ("name_len", "<i4"), ("part", "<u4"), ("total", "<u4"), ("fsize", "<u4"), ("fcrc", "<u4"),
                      ("dlen", "<u4"), ("pcrc", "<u4"), ("calc_crc", "<u4"), ("reserved", "<u4")])
assert FRAME_REC.itemsize == 64
DTYPES = {np.dtype(np.float32): DTYPE_F32, np.dtype(np.float64): DTYPE_F64, np.dtype(np.int16): DTYPE_I16}

# every symbol include/amr.h declares (tests/test_abi.py checks the export table)
EXPORTS = [
    "amr_abi_version", "amr_build_id", "amr_last_error", "amr_device_count", "amr_set_device", "amr_malloc", "amr_free",
    "amr_memcpy_h2d", "amr_memcpy_d2h", "amr_memcpy_d2d", "amr_device_synchronize",
    "amr_psk_plan_create", "amr_psk_plan_destroy", "amr_psk_plan_out_capacity", "amr_psk_plan_scratch_bytes",
    "amr_psk_plan_bytes_estimate", "amr_fsk_plan_bytes_estimate",
    "amr_psk_plan_synchronize", "amr_psk_plan_enable_timing", "amr_psk_plan_timings", "amr_psk_plan_set_inflight",
    "amr_psk_plan_exact_streams", "amr_psk_demod_host", "amr_psk_demod_device", "amr_psk_demod_fec_device",
    "amr_psk_slice_host", "amr_psk_plan_last_layout", "amr_synth_tile_noise",
    "amr_psk_demod_host_async", "amr_fsk_demod_host_async", "amr_host_register", "amr_host_unregister",
    "amr_host_alloc", "amr_host_free",
    "amr_fsk_plan_create", "amr_fsk_plan_destroy", "amr_fsk_plan_out_capacity", "amr_fsk_plan_scratch_bytes",
    "amr_fsk_plan_resident_bytes",
    "amr_fsk_plan_fft_length", "amr_fsk_plan_live_columns", "amr_fsk_plan_synchronize", "amr_fsk_plan_enable_timing", "amr_fsk_plan_timings",
    "amr_fsk_demod_host", "amr_fsk_demod_device", "amr_fsk_envelopes_host", "amr_fft_c2c_host", "amr_hilbert_host",
    "amr_fec_decode_host", "amr_frame_parse_host", "amr_frame_parse_device", "amr_comm_unique_id", "amr_comm_create", "amr_comm_destroy", "amr_allgather", "amr_fsk_allgather",
    "amr_comm_synchronize", "amr_comm_allgather_host", "amr_comm_allreduce_max", "amr_comm_world", "amr_tx_samples", "amr_tx_work_bytes", "amr_modulate_host", "amr_modulate_device",
    "amr_resample_host", "amr_hilbert_env_exact_host", "amr_fsk_plan_exact_streams",
    "amr_fsk_plan_set_exact_mode", "amr_psk_plan_set_layout", "amr_psk_plan_split_info", "amr_psk_split_design",
    "amr_psk_split_symbols_host", "amr_psk_f32_margin", "amr_psk_plan_last_f32f", "amr_split_state_tables",
    "amr_psk_plan_split_conv",
    "amr_fsk_plan_set_layout", "amr_fsk_plan_split_info", "amr_fsk_split_design", "amr_fsk_split_bandpass_host",
    "amr_fsk_fft_margin", "amr_fsk_plan_margin", "amr_fsk_plan_set_split_strict", "amr_fsk_plan_split_strict",
    "amr_fsk_plan_last_strict", "amr_fsk_split_strict_design", "amr_fsk_split_bounds_host",
    "amr_fsk_plan_split_conv",
    "amr_psk_demod_host_edges", "amr_psk_demod_device_edges", "amr_fsk_demod_host_edges", "amr_fsk_demod_device_edges",
    "amr_psk_split_bounds_host", "amr_psk_plan_set_split_strict", "amr_psk_plan_split_strict",
    "amr_psk_plan_last_strict", "amr_psk_split_strict_design",
]

TX_BPSK, TX_QPSK, TX_FSK = 0, 1, 2
TX_MODES = {"bpsk": TX_BPSK, "qpsk": TX_QPSK, "fsk": TX_FSK}


def tx_samples(mode: int, n_bytes: int, baud, samp_rate) -> int:
    """len() of the reference modulator's output for an n_bytes payload."""
    n = lib().amr_tx_samples(mode, n_bytes, float(baud), float(samp_rate))
    if n < 0:
        _raise_tx(int(n))
    return int(n)


def _raise_tx(rc: int):
    msg = lib().amr_last_error().decode("utf-8", "replace")
    if msg.startswith("could not broadcast"):
        raise ValueError(msg)                      # numpy's error, modem.py:58-61 / 181-183
    if msg == "float division by zero":
        raise ZeroDivisionError(msg)
    raise AmrError(rc, msg)


def modulate(mode: int, datas, baud, f0, f1=0.0, samp_rate=96000, n_out=None, pcm=False):
    """Batched transmit side on the GPU (amr_modulate_host): the reference
    modulator's float32 waveform of every payload in `datas` (modem.py:28-65,
    138-186, 270-295), cut / zero-padded to n_out samples (default: the
    longest natural length).  pcm=True also returns wav_from_array's int16."""
    require_gpu()
    n = len(datas)
    lens = np.array([len(d) for d in datas], np.int64)
    if n_out is None:
        n_out = max((tx_samples(mode, int(x), baud, samp_rate) for x in lens), default=0)
    stride = max(1, int(lens.max()) if n else 1)
    buf = np.zeros((max(n, 1), stride), np.uint8)
    for i, d in enumerate(datas):
        buf[i, :len(d)] = np.frombuffer(bytes(d), np.uint8)
    out = np.zeros((n, n_out), np.float32)
    pc = np.zeros((n, n_out), np.int16) if pcm else None
    rc = lib().amr_modulate_host(mode, float(baud), float(f0), float(f1), float(samp_rate), ptr(buf), stride,
                                 ptr(lens), n, ptr(out), n_out, n_out, ptr(pc) if pcm else None, n_out)
    if rc != AMR_OK:
        _raise_tx(rc)
    return (out, pc) if pcm else out


def psk_slice(kind: str, sym: np.ndarray) -> np.ndarray:
    """The slicer stage alone on the GPU (K4a): sym [B][S] complex128 -> the
    decided bits [B][bits] as uint8 (modem.py:214-241 QPSK, :100-105 BPSK)."""
    require_gpu()
    sym = np.ascontiguousarray(np.atleast_2d(sym), np.complex128)
    B, S = sym.shape
    nbits = max(0, (S - 1) * (2 if kind == "qpsk" else 1))
    nw = max(1, (nbits + 31) // 32)
    words = np.zeros((B, nw), np.uint32)
    check(lib().amr_psk_slice_host(PSK_QPSK if kind == "qpsk" else PSK_BPSK, ptr(sym), B, S, ptr(words)))
    bits = np.unpackbits(words.astype(">u4").view(np.uint8).reshape(B, -1), axis=1)
    return bits[:, :nbits]


def frame_parse(raws, max_cands: int = 64):
    """Batched decoder.parse_fbp_stream_enhanced scan (decoder.py:142-208) on
    the GPU: for each bytes object, (n_candidates, records[:min(n, max_cands)])
    with the reference's per-candidate verdict (FRAME_*) and header fields."""
    require_gpu()
    n = len(raws)
    if n == 0:
        return []
    lens = np.array([len(r) for r in raws], np.int64)
    stride = max(1, int(lens.max()))
    buf = np.zeros((n, stride), np.uint8)
    for i, r in enumerate(raws):
        buf[i, :len(r)] = np.frombuffer(r, np.uint8)
    cnt = np.zeros(n, np.int32)
    recs = np.zeros((n, max_cands), FRAME_REC)
    check(lib().amr_frame_parse_host(ptr(buf), stride, ptr(lens), n, max_cands, ptr(cnt), recs.ctypes.data))
    return [(int(cnt[i]), recs[i, :min(int(cnt[i]), max_cands)]) for i in range(n)]


class PinnedArray:
    """A numpy array over page-locked host memory (amr_host_alloc): the buffer
    a capture loop fills and hands to the *_demod_host_async entries."""

    def __init__(self, shape, dtype):
        self.nbytes = int(np.prod(shape)) * np.dtype(dtype).itemsize
        self._p = ctypes.c_void_p()
        check(lib().amr_host_alloc(ctypes.byref(self._p), max(1, self.nbytes)))
        buf = (ctypes.c_uint8 * max(1, self.nbytes)).from_address(self._p.value)
        self.array = np.frombuffer(buf, dtype=dtype, count=int(np.prod(shape))).reshape(shape)

    def close(self):
        if self._p:
            self.array = None
            lib().amr_host_free(self._p)
            self._p = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class AmrError(RuntimeError):
    """A libamr.so call failed (message from amr_last_error)."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"libamr error {code}: {msg}")
        self.code = code


_lib = None
_lib_lock = threading.Lock()
P, I64, I32, D, F = ctypes.c_void_p, ctypes.c_int64, ctypes.c_int, ctypes.c_double, ctypes.c_float


def lib():
    """Load libamr.so (raises if it was never built -- there is no fallback)."""
    global _lib
    with _lib_lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise AmrError(AMR_E_NODEVICE, f"{LIB_PATH} not found: build it with "
                                           "`python audio-modem-radio_amd/build.py` (there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        sig = {
            "amr_abi_version": (I32, []),
            "amr_build_id": (ctypes.c_char_p, []),
            "amr_last_error": (ctypes.c_char_p, []),
            "amr_device_count": (I32, [P]),
            "amr_set_device": (I32, [I32]),
            "amr_malloc": (I32, [P, I64]),
            "amr_free": (I32, [P]),
            "amr_memcpy_h2d": (I32, [P, P, I64]),
            "amr_memcpy_d2h": (I32, [P, P, I64]),
            "amr_memcpy_d2d": (I32, [P, P, I64]),
            "amr_device_synchronize": (I32, []),
            "amr_psk_plan_create": (I32, [P, I32, I32, I64, I64, I64, P, P, P, I32, P, P, P, I32, P, I64]),
            "amr_psk_plan_destroy": (I32, [P]),
            "amr_psk_plan_out_capacity": (I64, [P]),
            "amr_psk_plan_scratch_bytes": (I64, [P]),
            "amr_psk_plan_bytes_estimate": (I64, [I32, I64, I64, I64, I32, I32, I64]),
            "amr_fsk_plan_bytes_estimate": (I64, [I64, I64, I32, I64]),
            "amr_psk_plan_synchronize": (I32, [P]),
            "amr_psk_plan_enable_timing": (I32, [P, I32]),
            "amr_psk_plan_set_inflight": (I32, [P, I32]),
            "amr_psk_plan_timings": (I32, [P, P, I32]),
            "amr_psk_plan_exact_streams": (I32, [P, P]),
            "amr_psk_demod_host": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_psk_demod_device": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_psk_demod_host_edges": (I32, [P, P, I32, I64, I64, P, P, I64, P, P]),
            "amr_psk_demod_device_edges": (I32, [P, P, I32, I64, I64, P, P, I64, P, P]),
            "amr_fsk_demod_host_edges": (I32, [P, P, I32, I64, I64, P, P, I64, P, P]),
            "amr_fsk_demod_device_edges": (I32, [P, P, I32, I64, I64, P, P, I64, P, P]),
            "amr_psk_split_bounds_host": (I32, [P, P, I32, I64, I64, P, P, P]),
            "amr_psk_plan_set_split_strict": (I32, [P, I32]),
            "amr_psk_plan_split_strict": (I32, [P]),
            "amr_psk_plan_last_strict": (I32, [P]),
            "amr_psk_split_strict_design": (I32, [P, P, P, I32, P, P, P, I32, I64, I64, I64, P, P]),
            "amr_psk_demod_fec_device": (I32, [P, P, I32, I64, I64, P, I64, P, P, P, I64, P, P]),
            "amr_psk_slice_host": (I32, [I32, P, I64, I64, P]),
            "amr_psk_plan_last_layout": (I32, [P]),
            "amr_psk_plan_set_layout": (I32, [P, I32]),
            "amr_psk_plan_split_info": (I32, [P, P, P, P, P, P]),
            "amr_psk_split_design": (I32, [P, P, I32, P, P, I32, I64, I64, P, P, P]),
            "amr_psk_split_symbols_host": (I32, [P, P, I32, I64, I64, I64, P]),
            "amr_split_state_tables": (I32, [P, P, P, I32, I64, P, P]),
            "amr_psk_plan_split_conv": (I32, [P]),
            "amr_psk_f32_margin": (D, [P, P, I32]),
            "amr_psk_plan_last_f32f": (I32, [P]),
            "amr_psk_demod_host_async": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_fsk_demod_host_async": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_host_register": (I32, [P, I64]),
            "amr_host_alloc": (I32, [P, I64]),
            "amr_host_free": (I32, [P]),
            "amr_host_unregister": (I32, [P]),
            "amr_synth_tile_noise": (I32, [P, I64, I64, P, I64, I64, F, ctypes.c_uint64]),
            "amr_fsk_plan_create": (I32, [P, I32, I64, I64, P, P, P, P, P, P, I32, I64]),
            "amr_fsk_plan_destroy": (I32, [P]),
            "amr_fsk_plan_out_capacity": (I64, [P]),
            "amr_fsk_plan_scratch_bytes": (I64, [P]),
            "amr_fsk_plan_resident_bytes": (I64, [P]),
            "amr_fsk_plan_fft_length": (I64, [P]),
            "amr_fsk_plan_live_columns": (I32, [P]),
            "amr_fsk_plan_synchronize": (I32, [P]),
            "amr_fsk_plan_enable_timing": (I32, [P, I32]),
            "amr_fsk_plan_timings": (I32, [P, P, I32]),
            "amr_fsk_demod_host": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_fsk_demod_device": (I32, [P, P, I32, I64, I64, P, I64, P, P]),
            "amr_fsk_envelopes_host": (I32, [P, P, I32, I64, I64, P, P]),
            "amr_fft_c2c_host": (I32, [P, P, I64, I64, I32, I32]),
            "amr_hilbert_host": (I32, [P, P, I64, I64, I32]),
            "amr_fec_decode_host": (I32, [P, I64, P, I64, P, I64, P, P]),
            "amr_frame_parse_host": (I32, [P, I64, P, I64, I64, P, P]),
            "amr_frame_parse_device": (I32, [P, P, I64, P, I64, I64, P, P]),
            "amr_comm_unique_id": (I32, [P]),
            "amr_comm_create": (I32, [P, P, I32, I32, I32]),
            "amr_comm_destroy": (I32, [P]),
            "amr_allgather": (I32, [P, P, P, I64, P]),
            "amr_fsk_allgather": (I32, [P, P, P, I64, P]),
            "amr_comm_synchronize": (I32, [P]),
            "amr_comm_allgather_host": (I32, [P, P, P, I64]),
            "amr_comm_allreduce_max": (I32, [P, P, I64]),
            "amr_comm_world": (I32, [P, P, P]),
            "amr_tx_samples": (I64, [I32, I64, D, D]),
            "amr_resample_host": (I32, [P, I64, I64, I64, P, I32]),
            "amr_hilbert_env_exact_host": (I32, [P, I64, I64, P, I32]),
            "amr_fsk_plan_exact_streams": (I32, [P, P]),
            "amr_fsk_plan_set_exact_mode": (I32, [P, I32]),
            "amr_fsk_plan_set_layout": (I32, [P, I32]),
            "amr_fsk_plan_split_info": (I32, [P, P, P, P, P, P]),
            "amr_fsk_split_design": (I32, [I64, P, P, P, P, I32, P, P, P]),
            "amr_fsk_fft_margin": (I32, [I64, P, P, P, P, P, P, I32, P]),
            "amr_fsk_plan_margin": (I32, [P, P, P]),
            "amr_fsk_plan_set_split_strict": (I32, [P, I32]),
            "amr_fsk_plan_split_strict": (I32, [P]),
            "amr_fsk_plan_last_strict": (I32, [P]),
            "amr_fsk_split_strict_design": (I32, [P, P, P, I32, I64, P, P]),
            "amr_fsk_split_bounds_host": (I32, [P, P, I32, I64, I64, P, P, P]),
            "amr_fsk_split_bandpass_host": (I32, [P, P, I32, I64, I64, I64, P]),
            "amr_fsk_plan_split_conv": (I32, [P]),
            "amr_tx_work_bytes": (I64, [I32, D, D, I64, I64]),
            "amr_modulate_host": (I32, [I32, D, D, D, D, P, I64, P, I64, P, I64, I64, P, I64]),
            "amr_modulate_device": (I32, [P, I32, D, D, D, D, P, I64, P, I64, P, I64, I64, P, I64, P, I64]),
        }
        for name, (res, args) in sig.items():
            fn = getattr(L, name)
            fn.restype = res
            fn.argtypes = args
        _lib = L
        return L


def check(rc: int):
    if rc != AMR_OK:
        raise AmrError(rc, lib().amr_last_error().decode("utf-8", "replace"))
    return rc


def ptr(a) -> ctypes.c_void_p:
    return ctypes.c_void_p(a.ctypes.data)


def is_kernel_dtype(dt) -> bool:
    """float32 / float64: the dtypes the kernels read and extend themselves."""
    return np.dtype(dt) in (np.dtype(np.float32), np.dtype(np.float64))


def raw_input(x: np.ndarray, pad: int):
    """A raw capture [B][n] of any other real dtype -- integers of every width
    (int16 as its values, not PCM), bool, float16, longdouble -- as the
    reference's filtfilt sees it (modem.py:77, 198, 308; scipy
    _arraytools.odd_ext): (xk, edges).  xk: the samples as float32 (exact for
    integers of <= 16 bits, bool, float16) or float64 (numpy's cast, which is
    lfilter's own); edges [B][2 pad] float64: the odd extension 2*x[0] - x[k]
    computed by numpy IN x's dtype -- integer wraparound, bool -> int64,
    float16 rounding -- the left pad then the right (include/amr.h
    amr_psk_demod_host_edges).  n > pad (the plan's design checked it)."""
    x = np.ascontiguousarray(x)
    if not x.dtype.isnative:
        x = np.ascontiguousarray(x.astype(x.dtype.newbyteorder("=")))
    pad = int(pad)
    with np.errstate(all="ignore"):                      # numpy warns where scipy would, e.g. float16 overflow
        left = 2 * x[:, :1] - x[:, pad:0:-1]             # ext index j < pad: 2 x[0] - x[pad - j]
        right = 2 * x[:, -1:] - x[:, -2:-(pad + 2):-1]    # ext index pad + n + r: 2 x[n-1] - x[n-2-r]
        edges = np.ascontiguousarray(np.concatenate([left, right], axis=1), np.float64)
    narrow = x.dtype.kind == "b" or (x.dtype.kind in "iu" and x.dtype.itemsize <= 2) or x.dtype == np.float16
    return np.ascontiguousarray(x, np.float32 if narrow else np.float64), edges


def device_count() -> int:
    n = ctypes.c_int(0)
    rc = lib().amr_device_count(ctypes.byref(n))
    return n.value if rc == AMR_OK else 0


def default_device() -> int:
    for k in ("AMR_DEVICE", "LOCAL_RANK"):
        if k in os.environ:
            return int(os.environ[k])
    return 0


def require_gpu():
    if device_count() < 1:
        raise AmrError(AMR_E_NODEVICE, "no GPU visible to libamr.so: the demodulator runs only on the "
                                       "MI355X (there is no CPU fallback)")


# ---------------------------------------------------------------------------
# filter design (host, scipy) -- exactly the reference's calls
def design_psk(kind: str, n: int, baud, carrier=3000.0, samp_rate=96000):
    """Return (sps, first, bp(b,a,zi), lp(b,a,zi), lo4) or raise scipy's ValueError.

    Order of the reference's failure points is kept: band-pass design,
    band-pass filtfilt padlen check, low-pass design (modem.py:76-88 / 197-204)."""
    from scipy import signal
    sps = int(samp_rate / baud)
    nyq = samp_rate / 2
    if kind == "qpsk":
        low = (carrier - baud * 1.5) / nyq
        high = (carrier + baud * 1.5) / nyq
        first = sps // 2
    else:
        low = (carrier - baud) / nyq
        high = (carrier + baud) / nyq
        first = sps
    b, a = signal.butter(4, [max(0.01, low), min(0.99, high)], btype="band")
    ntaps = max(len(a), len(b))
    if n <= 3 * ntaps:
        raise ValueError("The length of the input vector x must be greater than padlen, which is %d." % (3 * ntaps))
    bl, al = signal.butter(4, baud / nyq, btype="low")
    bp = tuple(np.ascontiguousarray(v, np.float64) for v in (b, a, signal.lfilter_zi(b, a)))
    lp = tuple(np.ascontiguousarray(v, np.float64) for v in (bl, al, signal.lfilter_zi(bl, al)))
    return sps, first, bp, lp, lo_table(n, carrier, samp_rate)


def split_design(kind: str, n: int, baud, carrier=3000.0, samp_rate=96000):
    """The time-split design (host arithmetic in libamr.so, no device): dict of
    warmup_bp, warmup_lp, kappa, or None when the filters do not allow it."""
    sps, first, bp, lp, _ = design_psk(kind, n, baud, carrier, samp_rate)
    S = max(0, (n - first + sps - 1) // sps)
    w1, w2 = ctypes.c_int64(), ctypes.c_int64()
    k = ctypes.c_double()
    rc = lib().amr_psk_split_design(ptr(bp[0]), ptr(bp[1]), len(bp[0]), ptr(lp[0]), ptr(lp[1]), len(lp[0]), n, S,
                                    ctypes.byref(w1), ctypes.byref(w2), ctypes.byref(k))
    return None if rc != 0 else {"warmup_bp": w1.value, "warmup_lp": w2.value, "kappa": k.value}


def state_tables(b, a, zi, w: int):
    """amr_split_state_tables for one DF-II-T filter: (K [w][nt-1], Z0 [w+1][nt-1])."""
    b, a, zi = (np.ascontiguousarray(v, np.float64) for v in (b, a, zi))
    K, Z0 = np.zeros((w, len(b) - 1)), np.zeros((w + 1, len(b) - 1))
    check(lib().amr_split_state_tables(ptr(b), ptr(a), ptr(zi), len(b), int(w), ptr(K), ptr(Z0)))
    return K, Z0


def split_state_tables(kind: str, n: int, baud, carrier=3000.0, samp_rate=96000):
    """The time-split band-pass's convolution tables (K [w1][8], Z0 [w1 + 1][8];
    libamr.so host arithmetic, amr_split_state_tables), or None without a design."""
    d = split_design(kind, n, baud, carrier, samp_rate)
    if d is None:
        return None
    _, _, bp, _, _ = design_psk(kind, n, baud, carrier, samp_rate)
    w = d["warmup_bp"]
    ns = len(bp[0]) - 1
    K, Z0 = np.zeros((w, ns)), np.zeros((w + 1, ns))
    check(lib().amr_split_state_tables(ptr(bp[0]), ptr(bp[1]), ptr(bp[2]), len(bp[0]), w, ptr(K), ptr(Z0)))
    return K, Z0


STRICT_CONSTS = ["g1x", "gmax", "hz", "tk", "zi_sum", "zb", "kx", "ky", "u2", "gam", "c3", "w1", "w2", "n_sym", "nw",
                 "nk", "nh", "ng", "nz", "k12_off", "w_tail", "k12_tail", "hs_tail", "tz_tail", "lp_tail", "lp_rad",
                 "ok", "kappa"]


def split_strict_design(kind: str, n: int, baud, carrier=3000.0, samp_rate=96000):
    """The strict bound's design (libamr.so host arithmetic, amr_psk_split_strict_design):
    dict of the constants and the tables kabs, z0abs, lpc, W, K12, HS, GS, TZ; None
    when the plan has no strict bound."""
    sps, first, bp, lp, _ = design_psk(kind, n, baud, carrier, samp_rate)
    c = np.zeros(32)
    args = [ptr(bp[0]), ptr(bp[1]), ptr(bp[2]), len(bp[0]), ptr(lp[0]), ptr(lp[1]), ptr(lp[2]), len(lp[0]), n, first,
            sps, ptr(c)]
    if lib().amr_psk_split_strict_design(*args, None) != 0:
        return None
    d = dict(zip(STRICT_CONSTS, c[:len(STRICT_CONSTS)].tolist()))
    sizes = [("kabs", int(d["w1"])), ("z0abs", int(d["w1"]) + 1), ("lpc", int(d["n_sym"])), ("W", int(d["nw"])),
             ("K12", int(d["nk"])), ("HS", int(d["nh"])), ("GS", int(d["ng"])), ("TZ", int(d["nz"]))]
    tabs = np.zeros(sum(k for _, k in sizes))
    check(lib().amr_psk_split_strict_design(*args, ptr(tabs)))
    o = 0
    for name, k in sizes:
        d[name] = tabs[o:o + k]
        o += k
    return d


def f32_margin(kind: str, n: int, baud, carrier=3000.0, samp_rate=96000) -> float:
    """The float32 hand-off's symbol error bound per unit max |f| (libamr.so, host arithmetic)."""
    _, _, _, lp, _ = design_psk(kind, n, baud, carrier, samp_rate)
    return float(lib().amr_psk_f32_margin(ptr(lp[0]), ptr(lp[1]), len(lp[0])))


def lo_table(n: int, carrier, samp_rate) -> np.ndarray:
    """[n][4]: lo_re, lo_im, -(0*lo_im), 0*lo_re with lo = exp(-1j*2*pi*fc*t) (modem.py:200-201).

    The last two columns are the addends numpy's complex multiply
    (filtered + 0j) * lo evaluates: re = fma(f, lo_re, -(0*lo_im)),
    im = fma(f, lo_im, 0*lo_re)."""
    t = np.arange(n) / samp_rate
    lo = np.exp(-1j * 2 * np.pi * carrier * t)
    out = np.empty((n, 4))
    out[:, 0] = lo.real
    out[:, 1] = lo.imag
    out[:, 2] = -(0.0 * lo.imag)
    out[:, 3] = 0.0 * lo.real
    return out


class PskPlan:
    """A device plan: coefficients + LO in HBM + scratch for max_streams streams."""

    def __init__(self, kind: str, n: int, baud, carrier=3000.0, samp_rate=96000, max_streams=64,
                 device=None):
        self.kind, self.n, self.baud, self.carrier, self.samp_rate = kind, n, baud, carrier, samp_rate
        self.sps, self.first, self.bp, self.lp, lo4 = design_psk(kind, n, baud, carrier, samp_rate)
        require_gpu()
        self.device = default_device() if device is None else device
        self.max_streams = int(max_streams)
        h = ctypes.c_void_p()
        b, a, zi = self.bp
        bl, al, zil = self.lp
        check(lib().amr_psk_plan_create(ctypes.byref(h), self.device, PSK_QPSK if kind == "qpsk" else PSK_BPSK,
                                        n, self.sps, self.first, ptr(b), ptr(a), ptr(zi), len(b),
                                        ptr(bl), ptr(al), ptr(zil), len(bl), ptr(lo4), self.max_streams))
        self.handle = h
        self.out_cap = int(lib().amr_psk_plan_out_capacity(h))
        self.lock = threading.Lock()

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            try:
                _lib.amr_psk_plan_destroy(h)
            except Exception:
                pass
            self.handle = None

    def demod_host(self, x: np.ndarray):
        """x [B][N] float32/float64/int16 (int16 = PCM read as int16/32768). Returns (list[bytes], sync)."""
        x = np.ascontiguousarray(x)
        dt = DTYPES
        B = x.shape[0]
        outs, syncs = [], np.empty(B, np.int64)
        cap = max(self.out_cap, 1)
        for s0 in range(0, B, self.max_streams):
            xb = x[s0:s0 + self.max_streams]
            nb = xb.shape[0]
            out = np.empty((nb, cap), np.uint8)
            ln = np.empty(nb, np.int64)
            sy = np.empty(nb, np.int64)
            with self.lock:
                check(lib().amr_psk_demod_host(self.handle, ptr(xb), dt[xb.dtype], nb, xb.shape[1], ptr(out), cap,
                                               ptr(ln), ptr(sy)))
            outs += [out[i, :ln[i]].tobytes() for i in range(nb)]
            syncs[s0:s0 + nb] = sy
        return outs, syncs

    def demod_host_raw(self, x: np.ndarray):
        """x [B][N] of a dtype the kernels do not store (raw_input): the
        reference's semantics for that array.  Returns (list[bytes], sync)."""
        xk, edges = raw_input(np.atleast_2d(x), 3 * len(self.bp[0]))
        B = xk.shape[0]
        outs, syncs = [], np.empty(B, np.int64)
        cap = max(self.out_cap, 1)
        for s0 in range(0, B, self.max_streams):
            xb, eb = xk[s0:s0 + self.max_streams], edges[s0:s0 + self.max_streams]
            nb = xb.shape[0]
            out = np.empty((nb, cap), np.uint8)
            ln = np.empty(nb, np.int64)
            sy = np.empty(nb, np.int64)
            with self.lock:
                check(lib().amr_psk_demod_host_edges(self.handle, ptr(xb), DTYPES[xb.dtype], nb, xb.shape[1],
                                                     ptr(eb), ptr(out), cap, ptr(ln), ptr(sy)))
            outs += [out[i, :ln[i]].tobytes() for i in range(nb)]
            syncs[s0:s0 + nb] = sy
        return outs, syncs

    def scratch_bytes(self) -> int:
        """Device bytes this plan holds (scratch + host-API staging)."""
        return int(lib().amr_psk_plan_scratch_bytes(self.handle)) if self.handle else 0

    def enable_timing(self, on=True):
        check(lib().amr_psk_plan_enable_timing(self.handle, 1 if on else 0))

    def set_inflight(self, batches: int):
        """Hint: `batches` batches are kept in flight at once, each on its own plan."""
        check(lib().amr_psk_plan_set_inflight(self.handle, int(batches)))

    def timings(self) -> dict:
        ms = (ctypes.c_float * len(T_NAMES))()
        check(lib().amr_psk_plan_timings(self.handle, ms, len(T_NAMES)))
        return {k: float(v) for k, v in zip(T_NAMES, ms) if v >= 0}

    LAYOUTS = {"row": 0, "lane": 1, "split": 2}

    def last_layout(self) -> str:
        """'row' (state-per-lane kernels), 'lane' (one stream per lane) or 'split'
        (time-split passes, margin-checked, serial fallback) for the last call."""
        return {v: k for k, v in self.LAYOUTS.items()}.get(int(lib().amr_psk_plan_last_layout(self.handle)), "?")

    def set_layout(self, layout):
        """Force 'row' / 'lane' / 'split' for this plan's calls; None: by streams in flight."""
        check(lib().amr_psk_plan_set_layout(self.handle, -1 if layout is None else self.LAYOUTS[layout]))

    def split_symbols(self, x: np.ndarray, chunk: int = 0) -> np.ndarray:
        """Diagnostic: the time-split passes' symbol samples [B][S] complex (not bit-exact)."""
        x = np.ascontiguousarray(np.atleast_2d(x))
        B = x.shape[0]
        S = max(0, (self.n - self.first + self.sps - 1) // self.sps)
        sym = np.zeros((B, S, 2))
        with self.lock:
            check(lib().amr_psk_split_symbols_host(self.handle, ptr(x), DTYPES[x.dtype], B, x.shape[1], int(chunk),
                                                    ptr(sym)))
        return sym[..., 0] + 1j * sym[..., 1]

    def set_split_strict(self, on):
        """The time-split layout's strict bound for this plan: True / False, None = the
        process default (AMR_PSK_SPLIT_STRICT=1)."""
        check(lib().amr_psk_plan_set_split_strict(self.handle, -1 if on is None else (1 if on else 0)))

    def split_strict(self) -> bool:
        return int(lib().amr_psk_plan_split_strict(self.handle)) == 1

    def last_strict(self) -> bool:
        return int(lib().amr_psk_plan_last_strict(self.handle)) == 1

    def split_bounds(self, x: np.ndarray):
        """Diagnostic: the strict passes' symbols [B][S] complex, the bound e [B][S] on each
        component's |split - reference|, and per stream (E1, F, X, P3) (P3 < 0: caps failed)."""
        x = np.ascontiguousarray(np.atleast_2d(x))
        B = x.shape[0]
        S = max(0, (self.n - self.first + self.sps - 1) // self.sps)
        sym = np.zeros((B, S, 2))
        eb = np.zeros((B, S))
        sc = np.zeros((B, 4))
        with self.lock:
            check(lib().amr_psk_split_bounds_host(self.handle, ptr(x), DTYPES[x.dtype], B, x.shape[1], ptr(sym),
                                                  ptr(eb), ptr(sc)))
        return sym[..., 0] + 1j * sym[..., 1], eb, sc

    def last_f32f(self) -> bool:
        """The last call handed the band-pass output to the low-pass in float32."""
        return int(lib().amr_psk_plan_last_f32f(self.handle)) == 1

    def split_conv(self) -> bool:
        """The time-split layout starts its band-pass chunks from convolution
        states (KS0) rather than warm-ups (AMR_PSK_SPLIT_CONV=0)."""
        return int(lib().amr_psk_plan_split_conv(self.handle)) == 1

    def split_info(self) -> dict:
        """The time-split layout: streams the last call flagged for the serial path
        (-1: that call ran another layout), warm-ups, chunk length, error bound kappa."""
        fl, w1, w2, L = (ctypes.c_int64() for _ in range(4))
        k = ctypes.c_double()
        check(lib().amr_psk_plan_split_info(self.handle, ctypes.byref(fl), ctypes.byref(w1), ctypes.byref(w2),
                                            ctypes.byref(L), ctypes.byref(k)))
        return {"flagged": fl.value, "warmup_bp": w1.value, "warmup_lp": w2.value, "chunk": L.value,
                "kappa": k.value}

    def exact_streams(self) -> int:
        c = ctypes.c_int64(0)
        check(lib().amr_psk_plan_exact_streams(self.handle, ctypes.byref(c)))
        return c.value


class PlanCache:
    """LRU of device plans bounded by the HBM they hold.

    The reference keeps no state between calls; a long-running receiver
    decoding captures of ever-different lengths (the live-capture path,
    filebeep_advanced_v2.py:324) must not accumulate one plan per length.
    Plans are kept while their summed device bytes (scratch_bytes(), incl.
    host-API staging) stay within `budget` and there are at most
    `max_entries` of them; the least recently used are dropped first (their
    HBM is released when the last caller holding one lets go of it)."""

    def __init__(self, budget_bytes: int, max_entries: int = 32):
        import collections
        self.budget = int(budget_bytes)
        self.max_entries = int(max_entries)
        self._d = collections.OrderedDict()
        self.lock = threading.Lock()

    def get(self, key, need: int, make, estimate=None):
        """The cached plan for key if it holds >= need streams, else make(need);
        before making it, plans are evicted until estimate(need) (the new
        plan's device bytes) fits beside the rest within the budget."""
        with self.lock:
            pl = self._d.get(key)
            if pl is not None and pl.max_streams >= need:
                self._d.move_to_end(key)
                return pl
            if pl is not None:
                del self._d[key]                    # too small: its scratch goes before the new one's
                pl = None
            self._evict(reserve=int(estimate(need)) if estimate else 0)
            pl = make(need)
            self._d[key] = pl
            self._evict(reserve=0, keep=key)
            return pl

    def total_bytes(self) -> int:
        with self.lock:
            return self._total_unlocked()

    def _total_unlocked(self) -> int:
        return sum(p.scratch_bytes() for p in self._d.values())

    def __len__(self):
        return len(self._d)

    def clear(self):
        with self.lock:
            self._d.clear()

    def _evict(self, reserve: int, keep=None):
        total = sum(p.scratch_bytes() for p in self._d.values())
        while self._d and (total + reserve > self.budget or len(self._d) > self.max_entries):
            k = next(iter(self._d))
            if k == keep:
                if len(self._d) == 1:
                    break
                self._d.move_to_end(k)
                k = next(iter(self._d))
            total -= self._d.pop(k).scratch_bytes()


def _cache_budget() -> int:
    return int(float(os.environ.get("AMR_PLAN_CACHE_BYTES", 64e9)))


def stream_bucket(batch: int, cap: int) -> int:
    """Plan size for a batch: the next power of two (a single-stream call gets
    a one-stream plan), capped at `cap` streams per launch."""
    b = max(1, min(int(batch), int(cap)))
    return 1 << (b - 1).bit_length()


# ONE plan cache for every demodulator (PSK and FSK plans, keyed by kind):
# its byte budget (AMR_PLAN_CACHE_BYTES, default 64 GB, 2/9 of an MI355X's
# HBM) bounds all the drop-in path's device memory together.
plan_cache = PlanCache(_cache_budget())
PSK_MAX_CHUNK = 4096


def get_psk_plan(kind: str, n: int, baud, carrier, samp_rate, batch: int) -> PskPlan:
    """Plan cache keyed by the reference call's parameters (and device)."""
    dev = default_device()
    key = ("psk", kind, int(n), float(baud), float(carrier), float(samp_rate), dev)
    need = stream_bucket(batch, PSK_MAX_CHUNK)
    sps = int(samp_rate / baud)
    first = sps // 2 if kind == "qpsk" else sps

    def estimate(m):
        return max(0, int(lib().amr_psk_plan_bytes_estimate(PSK_QPSK if kind == "qpsk" else PSK_BPSK, int(n), sps,
                                                            first, 9, 5, m)))
    return plan_cache.get(key, need, lambda m: PskPlan(kind, n, baud, carrier, samp_rate, max_streams=m, device=dev),
                          estimate if sps >= 1 else None)


def fec_decode_host(datas):
    """Batched fec.ReedSolomonFEC.decode on the GPU. Returns (list[bytes], crc_ok[list[bool]])."""
    require_gpu()
    datas = [bytes(d) for d in datas]
    n = len(datas)
    if n == 0:
        return [], []
    stride = max(1, max(len(d) for d in datas))
    buf = np.zeros((n, stride), np.uint8)
    ln = np.array([len(d) for d in datas], np.int64)
    for i, d in enumerate(datas):
        buf[i, :len(d)] = np.frombuffer(d, np.uint8)
    out = np.zeros((n, stride), np.uint8)
    out_len = np.zeros(n, np.int64)
    ok = np.zeros(n, np.int32)
    check(lib().amr_set_device(default_device()))
    check(lib().amr_fec_decode_host(ptr(buf), stride, ptr(ln), n, ptr(out), stride, ptr(out_len), ptr(ok)))
    return [out[i, :out_len[i]].tobytes() for i in range(n)], [bool(v) for v in ok]


def fft(x: np.ndarray, inverse: bool = False) -> np.ndarray:
    """numpy.fft.fft / ifft along the last axis of a [batch][n] complex array, on the GPU."""
    require_gpu()
    x = np.ascontiguousarray(np.atleast_2d(x), np.complex128)
    out = np.empty_like(x)
    check(lib().amr_fft_c2c_host(ptr(x), ptr(out), x.shape[1], x.shape[0], 1 if inverse else 0, default_device()))
    return out


def hilbert(x: np.ndarray) -> np.ndarray:
    """scipy.signal.hilbert(x) along the last axis of a real [batch][n] array, on the GPU."""
    require_gpu()
    x = np.ascontiguousarray(np.atleast_2d(x), np.float64)
    out = np.empty(x.shape, np.complex128)
    check(lib().amr_hilbert_host(ptr(x), ptr(out), x.shape[1], x.shape[0], default_device()))
    return out


def hilbert_env_exact(x: np.ndarray) -> np.ndarray:
    """np.abs(scipy.signal.hilbert(x)) along the last axis of a real [batch][n]
    array on the GPU, bit for bit (pocketfft's own transforms and numpy's
    complex arithmetic restated -- the FSK exact path's envelope stage)."""
    require_gpu()
    x = np.array(np.atleast_2d(x), np.float64, copy=True, order="C")
    out = np.empty_like(x)
    check(lib().amr_hilbert_env_exact_host(ptr(x), x.shape[1], x.shape[0], ptr(out), default_device()))
    return out


def resample(x: np.ndarray, num: int) -> np.ndarray:
    """scipy.signal.resample(x, num) for real float64 input (1-D, or rows of a
    2-D array resampled along the last axis) on the GPU, bit for bit
    (pocketfft's rfft / irfft restated) -- the resample of
    decoder.decode_wav_file (decoder.py:385-387)."""
    require_gpu()
    a = np.asarray(x)
    if a.dtype != np.float64:
        raise TypeError("resample: float64 input only (decode_wav_file's soundfile data)")
    rows = np.ascontiguousarray(np.atleast_2d(a))
    if rows.ndim != 2 or num < 1 or rows.shape[1] < 1:
        raise ValueError("resample: need 1-D / 2-D input with at least one sample and num >= 1")
    out = np.empty((rows.shape[0], int(num)), np.float64)
    check(lib().amr_resample_host(ptr(rows), rows.shape[1], int(num), rows.shape[0], ptr(out), default_device()))
    return out[0] if a.ndim == 1 else out
