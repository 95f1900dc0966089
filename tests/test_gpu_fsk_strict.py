"""The FSK split F1's STRICT margin on the MI355X (round 6).

A split call's F2 margin is tau + F ||ifft(h)||_1 / peak, F a bound per tone
on |z_split - z_serial| that holds for every input (fsk_kernels.hip FS0-FS2
step bounds, KF1-KF2; split_strict.h strict_design_bp per tone) -- the
default since round 6 (AMR_FSK_SPLIT_STRICT=0 / amr_fsk_plan_set_split_strict
keeps round 5's kappa margin).  Checked here: the device's per-tone maxima
and F are the numpy restatement's (tests/_util.py strict_pass_bounds over
oracle.fsk_split_stats -- tests/test_split_margin.py shows that restatement
>= the measured error on the CPU), F >= the device's own |split - serial| on
every sample, and strict calls give the reference's bytes."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

CASES = [(96000, 9600, 12000.0, 24000.0), (48000, 1200, 2400.0, 4800.0), (30000, 2400, 11229.28, 29833.37),
         (96000, 4800, 7000.0, 19000.0)]


def _signals(n, baud, mark, space, seed):
    import synth
    rng = np.random.default_rng(seed)
    t = np.arange(n) / 96000.0
    out = [rng.normal(0, 0.3, n), np.sign(np.sin(2 * np.pi * mark * t)), np.sin(2 * np.pi * space * t)]
    for _ in range(3):
        w = synth.fsk_waveform(synth.random_frame(rng, 100), baud, mark, space, 96000.0)
        x = np.zeros(n)
        x[:min(n, w.size)] = w[:n]
        out.append(x + rng.normal(0, 0.05, n))
    out.append(np.clip(4 * out[-1], -1, 1))
    return np.stack(out).astype(np.float32)


@pytest.mark.parametrize("n,baud,mark,space", CASES, ids=lambda v: str(v))
def test_device_bound_is_the_restatement_and_holds(n, baud, mark, space):
    import _amr
    import _fsk
    from oracle import oracle
    from _util import pass1_peak, strict_pass_bounds
    x = _signals(n, baud, mark, space, baud + n)
    sd = _fsk.split_design(n, baud, mark, space)
    D = _fsk.split_strict_design(n, baud, mark, space)
    assert sd is not None and D is not None
    _, tones = _fsk.design_fsk(n, baud, mark, space, 96000.0)
    T = [_amr.state_tables(b, a, zi, sd["warmup"]) for b, a, zi in tones]
    pl = _fsk.FskPlan(n, baud, mark, space, max_streams=x.shape[0])
    z, bnd, pk = pl.split_bounds(x)
    L = pl.split_info()["chunk"]
    assert L % 16 == 0
    ratio = []
    for i in range(x.shape[0]):
        p1 = pass1_peak(x[i], 21)
        assert pk[i] == p1, (i, pk[i], p1)
        for t, (b, a, zi) in enumerate(tones):
            want = oracle.split_filtfilt(b, a, x[i], L, sd["warmup"], tables=T[t])
            assert np.array_equal(z[i, :, t], want), (i, t)
            st = oracle.fsk_split_stats(x[i], b, a, L, sd["warmup"], T[t], D[t])
            pb = strict_pass_bounds(st, D[t], p1, n, L, 21)
            for slot, v in ((0, st["D1max"]), (2, st["y1max"]), (3, st["D2max"])):
                assert bnd[i, t, slot] == v, (i, t, slot, bnd[i, t, slot], v)
            assert np.isclose(bnd[i, t, 1], pb["E1max"], rtol=1e-9, atol=0), (i, t)
            assert np.isclose(bnd[i, t, 6], pb["Fmax"], rtol=1e-9, atol=0), (i, t)
            assert pb["ok"]
            act = float(np.abs(z[i, :, t] - oracle.filtfilt(b, a, x[i])).max())
            assert act <= bnd[i, t, 6], (i, t, act, bnd[i, t, 6])
            ratio.append(bnd[i, t, 6] / max(act, 1e-300))
    print(f"fsk@{baud} n={n}: device F / measured >= {min(ratio):.1f} over {len(ratio)} (stream, tone)")


def test_strict_default_bytes_and_flags():
    """One-capture calls on the benchmark's noisy FSK9600 captures with the
    strict margin (the default) and with round 5's kappa margin: bytes ==
    the oracle's both ways, the strict mode reported, the exact-path counts
    printed."""
    import _fsk
    import modem
    import synth
    from oracle import oracle
    n, B = 96000, 64
    x = synth.fsk_batch(B, n, 9600, 12000.0, 24000.0, seed=5, distinct=B, noise=0.05)
    want = [oracle.fsk_demodulate(x[i], 9600, 12000.0, 24000.0) for i in range(B)]
    pl = _fsk.get_fsk_plan(n, 9600, 12000.0, 24000.0, 96000, 1)
    assert pl.split_strict()
    exact = {}
    for strict in (True, False):
        pl.set_split_strict(strict)
        e = 0
        for i in range(B):
            got = modem.fsk_demodulate(x[i], baud=9600, mark_freq=12000.0, space_freq=24000.0)
            assert got == want[i], (strict, i)
            assert pl.split_info()["last_split"] and pl.last_strict() == strict
            e += pl.exact_streams()
        exact[strict] = e
    pl.set_split_strict(None)
    print(f"exact-path captures of {B}: strict {exact[True]}, kappa margin {exact[False]}")


def test_kappa_margin_golden_and_sweep(golden, sweep_golden):
    """Every golden and reference-sweep FSK case through the drop-in with the
    strict margin OFF (AMR_FSK_SPLIT_STRICT=0 in a subprocess: the default is
    read once per process) -- the round-5 path stays the reference's; the
    default (strict) runs through every other GPU test."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    code = f'''
import sys, json, numpy as np
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import modem, _fsk, _amr
from _util import call_case, call_sweep_case, expected, outcome
g = {os.path.join(here, "golden")!r}
m = json.load(open(g + "/manifest.json")); inp = np.load(g + "/inputs.npz")
bad = [c["id"] for c in m["cases"] if c["fn"].startswith("fsk")
       and outcome(lambda: call_case(modem, c, inp[c["id"]])) != expected(c)]
m = json.load(open(g + "/sweep_manifest.json")); inp = np.load(g + "/sweep.npz")
for c in m["cases"]:
    if c["fn"] != "fsk":
        continue
    x = inp[c["id"]]
    x = x.astype(np.float64) / 32768.0 if x.dtype == np.int16 else x
    if outcome(lambda: call_sweep_case(modem, c, x)) != expected(c):
        bad.append(c["id"])
strict = [p.split_strict() for p in _amr.plan_cache._d.values() if isinstance(p, _fsk.FskPlan)]
print("BAD", bad, "STRICT", any(strict), len(strict))
'''
    env = dict(os.environ, AMR_FSK_SPLIT_STRICT="0")
    r = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:]
    line = [ln for ln in r.stdout.splitlines() if ln.startswith("BAD")][-1]
    assert line.startswith("BAD [] STRICT False"), line
