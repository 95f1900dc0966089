"""Shared test helpers: run a golden case through a demod callable."""
from __future__ import annotations


def call_case(mod, case, x):
    """Dispatch one manifest case to `mod` (the product modem module or the oracle)."""
    fn, p = case["fn"], case["params"]
    if fn == "qpsk_demodulate":
        return mod.qpsk_demodulate(x, **p)
    if fn == "bpsk_demodulate":
        return mod.bpsk_demodulate(x, **p)
    if fn == "psk8_demodulate":
        return mod.psk8_demodulate(x, p["b"])
    if fn == "ofdm_demodulate_simple":
        return mod.ofdm_demodulate_simple(x, p["baud"], p["carrier"], p["num_subcarriers"])
    if fn == "fsk_demodulate":
        return mod.fsk_demodulate(x, **p)
    if fn == "fsk_high_speed_demodulate":
        return mod.fsk_high_speed_demodulate(x, p["baud"])
    raise KeyError(fn)


def outcome(fn):
    try:
        return ("ok", fn().hex())
    except ValueError as e:   # the reference's error contract is scipy's ValueError
        return ("err", "ValueError", str(e))


def expected(case):
    if case["status"] == "ok":
        return ("ok", case["out"])
    return ("err", case["etype"], case["emsg"])


def call_sweep_case(mod, case, x):
    """Dispatch one sweep case (tests/golden/sweep_manifest.json) to `mod`."""
    fn, p = case["fn"], case["params"]
    if fn == "fsk":
        return mod.fsk_demodulate(x, baud=p["baud"], mark_freq=p["f0"], space_freq=p["f1"], samp_rate=p["samp_rate"])
    f = mod.qpsk_demodulate if fn == "qpsk" else mod.bpsk_demodulate
    return f(x, baud=p["baud"], carrier=p["f0"], samp_rate=p["samp_rate"])


def fsk_device_demod(pl, x):
    """amr_fsk_demod_device on x copied to device memory: (bytes list, sync)."""
    import ctypes

    import numpy as np
    import _amr
    L = _amr.lib()
    B, n = x.shape
    cap = max(pl.out_cap, 1)
    ptrs = {}
    for name, nbytes in (("x", x.nbytes), ("out", B * cap), ("len", B * 8), ("sync", B * 8)):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), nbytes))
        ptrs[name] = p
    try:
        _amr.check(L.amr_memcpy_h2d(ptrs["x"], _amr.ptr(x), x.nbytes))
        _amr.check(L.amr_fsk_demod_device(pl.handle, ptrs["x"], _amr.DTYPES[x.dtype], B, n, ptrs["out"], cap,
                                          ptrs["len"], ptrs["sync"]))
        _amr.check(L.amr_fsk_plan_synchronize(pl.handle))
        out, ln, sy = np.empty((B, cap), np.uint8), np.empty(B, np.int64), np.empty(B, np.int64)
        for name, h in (("out", out), ("len", ln), ("sync", sy)):
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(h), ptrs[name], h.nbytes))
    finally:
        for p in ptrs.values():
            L.amr_free(p)
    return [out[i, :ln[i]].tobytes() for i in range(B)], sy


def pass1_peak(x, pad1=27) -> float:
    """The band-pass pass-1 input's peak: max |x| over the capture and its
    odd extension (formed in x's dtype, oracle.odd_edges) -- the peak the
    device's strict bound scales its caps by (an edge can reach 3 peak|x|)."""
    import numpy as np
    from oracle import oracle
    return float(max(np.abs(np.asarray(x, dtype=np.float64)).max(), np.abs(oracle.odd_edges(x, pad1)).max()))


def strict_pass_bounds(st, d, peak1, n, L, pad1):
    """The strict bound of a split filtfilt band-pass (psk_split_kernels.hip
    KB1-KB2 / fsk_kernels.hip KF1-KF2, restated in numpy) from its statistics
    st (oracle.psk_split_stats / fsk_split_stats) and design d: E1 / E2 per
    forward block, their maxima, the caps and whether they hold."""
    import numpy as np
    u, eta, two = 2.0 ** -53, 2.0 ** -1060, 2.0 + 2.0 ** -20
    BS = 16
    m1 = n + 2 * pad1
    nb1, LB = -(-m1 // BS), L // BS
    d1, d2, ds1, ds2 = st["d1"], st["d2"], st["ds1"], st["ds2"]
    D1m, y1m, D2m, fm0 = st["D1max"], st["y1max"], st["D2max"], st["fmax"]
    cap1 = 2.0 ** -10 * peak1
    p2 = y1m + cap1
    cap2 = 2.0 ** -10 * p2
    sec1 = d["u2"] * d["zb"] * cap1 + d["ky"] * cap1
    c1 = d["g1x"] * (sec1 + 2 * eta) + d["gmax"] * u * d["zi_sum"] * peak1
    W, K12, HS, GS, TZ = d["W"], d["K12"], d["HS"], d["GS"], d["TZ"]
    R1 = np.convolve(d1, W)[:nb1] + d["w_tail"] * D1m
    J = np.arange(nb1)
    c = J // LB
    q = J - c * LB
    gs = np.where(q < 64, GS[np.minimum(q, 63)], d["gmax"])
    S1 = np.where(c > 0, gs * (ds1[c] + d["tk"] * peak1), 0.0)
    E1 = two * R1 + c1 + S1
    E1max, S1max = E1.max(), S1.max()
    E1last = max(E1[-1], E1[-2] if nb1 > 1 else 0.0)
    sec2 = d["u2"] * d["zb"] * cap2 + d["kx"] * E1max + d["ky"] * cap2
    c2 = d["hz"] * c1 + d["g1x"] * (sec2 + 2 * eta) + 2.0 * d["gmax"] * u * d["zi_sum"] * p2
    # own2 over backward blocks
    R2 = np.convolve(d2, W)[:nb1] + d["w_tail"] * D2m
    c2b = J // LB
    q2 = J - c2b * LB
    gs2 = np.where(q2 < 64, GS[np.minimum(q2, 63)], d["gmax"])
    own2 = two * R2 + np.where(c2b > 0, gs2 * (ds2[c2b] + d["tk"] * p2), 0.0)
    off = int(d["k12_off"])
    A = np.full(nb1, d["k12_tail"] * D1m)
    for kq in range(K12.size):
        db = kq - off
        lo, hi = max(0, -db), min(nb1, nb1 - db)
        if lo < hi:
            A[lo:hi] += K12[kq] * d1[lo + db:hi + db]
    H = np.full(nb1, d["hs_tail"] * S1max)
    for db in range(HS.size):
        if db < nb1:
            H[:nb1 - db] += HS[db] * S1[db:]
    jhi = np.minimum(16 * J + 15, m1 - 1)
    Ka, Kb = (m1 - 1 - jhi) // BS, (m1 - 1 - 16 * J) // BS
    tzw = lambda k: np.where(k < TZ.size, TZ[np.minimum(k, TZ.size - 1)], d["tz_tail"])  # noqa: E731
    tz = np.maximum(tzw(Ka), tzw(Kb)) * E1last
    o2 = np.maximum(own2[np.clip(Ka, 0, nb1 - 1)], own2[np.clip(Kb, 0, nb1 - 1)])
    E2 = two * A + H + tz + o2 + c2
    Fmax = E2.max()
    return dict(E1=E1, E2=E2, E1max=E1max, Fmax=Fmax, cap1=cap1, cap2=cap2, fm0=st["fmax"],
                ok=bool(E1max <= cap1 and Fmax <= cap2))


def strict_symbol_bounds(st, d, peak1, n, first, sps, L, pad1=27, pad2=15):
    """The strict mode's per-symbol bound e(k) on |split - reference| of the
    complex symbol (psk_split_kernels.hip KB, restated in numpy) from a
    stream's split statistics st (oracle.psk_split_stats / the device's) and
    the design d (_amr.split_strict_design); peak1 = pass1_peak(x).  Returns (e [S], (E1max, Fmax,
    Xmax, P3, ok))."""
    import numpy as np
    BS = 16
    pb = strict_pass_bounds(st, d, peak1, n, L, pad1)
    E2, E1max, Fmax = pb["E2"], pb["E1max"], pb["Fmax"]
    nbs = -(-n // BS)
    fm = pb["fm0"] + Fmax
    fb = np.arange(nbs)
    ilo, ihi = 16 * fb, np.minimum(16 * fb + 15, n - 1)
    Fb = np.maximum(E2[(ilo + pad1) // BS], E2[(ihi + pad1) // BS])
    X = Fb * (1 + 2.0 ** -50) + 2.0 ** -52 * 1.0078125 * fm
    Xmax = X.max()
    P3 = 3.0 * (fm + Xmax)
    ok = pb["ok"]
    S = d["lpc"].size
    t = first + np.arange(S) * sps
    lo = t - int(d["lp_rad"]) - pad2
    hi = t + int(d["lp_rad"]) + pad2
    flo = np.where(lo > 0, lo // BS, 0)
    fhi = np.minimum(hi, n - 1) // BS
    xw = np.array([max(X[0], X[-1], X[a:b + 1].max()) for a, b in zip(flo, fhi)])
    # the symbol's complex error: the band-pass error through the unit-modulus
    # mixer and the real low-pass as one complex sum, sqrt2 on the
    # per-component roundings (the mixer's rho, the low-pass's c3 P3)
    rho = 2.0 ** -52 * 1.0078125 * fm
    t1 = np.sqrt(2.0) * ((d["lpc"] + d["lp_tail"]) * rho + d["c3"] * P3)
    e = (1 + 2.0 ** -30) * ((d["lpc"] * xw + d["lp_tail"] * Xmax) * (1 + 2.0 ** -50) + t1)
    return e, (E1max, Fmax, Xmax, P3, ok)
