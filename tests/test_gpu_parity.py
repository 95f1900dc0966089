"""GPU parity: the HIP path (through the C ABI) against the reference's own
outputs (golden fixtures) and against the oracle on seeded inputs up to the
BASELINE sizes.  Bar: bit-exact bytes (and identical error contracts)."""
import contextlib
import io
import os

import numpy as np
import pytest

from _util import call_case, expected, outcome

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def test_every_golden_psk_case_bit_exact(golden):
    import modem
    manifest, inputs = golden
    bad = []
    for case in manifest["cases"]:
        if case["fn"].startswith("fsk"):
            continue
        got = outcome(lambda: call_case(modem, case, inputs[case["id"]]))
        if got != expected(case):
            bad.append(case["id"])
    assert not bad, f"GPU differs from the reference on {bad}"


def test_golden_qpsk9600_as_one_batch(golden):
    import modem
    manifest, inputs = golden
    cases = [c for c in manifest["cases"] if c["id"].startswith("qpsk9600_f32_")]
    x = np.stack([inputs[c["id"]] for c in cases])
    outs = modem.qpsk_demodulate_batch(x, baud=9600)
    assert [o.hex() for o in outs] == [c["out"] for c in cases]


def test_exact_complex_lowpass_path_matches(golden, monkeypatch):
    """Force every stream through k_lowpass_exact (scipy's complex lfilter
    semantics) and check it reproduces the reference too."""
    import _amr
    manifest, inputs = golden
    monkeypatch.setenv("AMR_FORCE_EXACT_LOWPASS", "1")
    bad = []
    for case in manifest["cases"]:
        if case["status"] != "ok" or case["fn"] not in ("qpsk_demodulate", "bpsk_demodulate"):
            continue
        x = inputs[case["id"]]
        kind = "qpsk" if case["fn"] == "qpsk_demodulate" else "bpsk"
        p = case["params"]
        plan = _amr.PskPlan(kind, x.size, p["baud"], p.get("carrier", 3000.0), 96000, max_streams=1)
        outs, _ = plan.demod_host(x[None, :])
        if outs[0].hex() != case["out"]:
            bad.append(case["id"])
    assert not bad, bad


def test_silence_cases_take_exact_path(golden):
    """Exactly-zero regions must be routed to the exact kernel by the detector."""
    import _amr
    manifest, inputs = golden
    x = inputs["qpsk_tail_silence"]
    plan = _amr.PskPlan("qpsk", x.size, 9600, max_streams=1)
    outs, _ = plan.demod_host(x[None, :])
    assert outs[0].hex() == [c for c in manifest["cases"] if c["id"] == "qpsk_tail_silence"][0]["out"]
    assert plan.exact_streams() == 1
    xs = inputs["qpsk9600_f32_0"]
    plan2 = _amr.PskPlan("qpsk", xs.size, 9600, max_streams=1)
    plan2.demod_host(xs[None, :])
    assert plan2.exact_streams() == 0


def test_int16_pcm_path_equals_float64_reference(golden):
    """AMR_DTYPE_I16 (PCM read as int16/32768) == the reference on the float64 it would see."""
    import _amr
    manifest, inputs = golden
    x = inputs["qpsk9600_wav"]
    q = np.round(x * 32768.0).astype(np.int16)
    assert np.array_equal(q.astype(np.float64) / 32768.0, x)
    plan = _amr.PskPlan("qpsk", x.size, 9600, max_streams=1)
    outs, _ = plan.demod_host(q[None, :])
    assert outs[0].hex() == [c for c in manifest["cases"] if c["id"] == "qpsk9600_wav"][0]["out"]


_BATCHES = {}


def _seeded_batch(kind, baud, B, N):
    """The seeded input of a batch test and the oracle's bytes + sync for it,
    built once per module (the full-size row and lane tests share them; the
    three full-size batches hold ~8 GB of host memory)."""
    import synth
    from oracle import oracle
    key = (kind, baud, B, N)
    if key not in _BATCHES:
        if kind == "qpsk" and baud == 19200:
            x = synth.dpsk8_batch(B, N, baud, seed=B, distinct=8 if B < 8192 else 64)
        elif kind == "qpsk":
            x = synth.qpsk_batch(B, N, baud, seed=B, distinct=8)
        else:
            x = np.stack([synth.fit(synth.bpsk_waveform(synth.random_frame(np.random.default_rng(i), 200), baud), N)
                          + np.random.default_rng(i).normal(0, 0.05, N).astype(np.float32) for i in range(B)])
        want, wsync = oracle.psk_demod_batch(kind, x, baud, n_threads=min(16, os.cpu_count() or 1))
        _BATCHES[key] = (x, want, wsync)
    return _BATCHES[key]


@pytest.mark.parametrize("kind,baud,B,N", [("qpsk", 9600, 4096, 96000), ("qpsk", 9600, 8192, 96000),
                                           ("qpsk", 19200, 257, 96000),
                                           ("bpsk", 1200, 130, 48000), ("qpsk", 2400, 65, 30001)])
def test_batch_vs_oracle(kind, baud, B, N):
    """Seeded batches up to the BASELINE config-2 size (and the 8192-stream
    single launch of configs 4/5 on one GPU), every stream checked against the
    oracle (bit-exact bytes and sync index).  One batch alone: the row layout."""
    import _amr
    x, want, wsync = _seeded_batch(kind, baud, B, N)
    plan = _amr.PskPlan(kind, N, baud, max_streams=B)
    got, gsync = plan.demod_host(x)
    assert plan.last_layout() == "row"
    mism = [i for i in range(B) if got[i] != want[i]]
    assert not mism, f"{len(mism)} streams differ, first {mism[:5]}"
    assert np.array_equal(gsync, wsync)


@pytest.mark.parametrize("baud", [9600, 19200])
def test_full_size_lane_layout_as_benched(baud):
    """Configs 4 (OFDM8 = the QPSK@9600 path, modem.py:375-376) and 5's demod
    (8PSK@19200 = the QPSK path, modem.py:348) at their full 8192 x 96000, in
    the layout bench.py times: a plan told 16 batches are in flight (so the
    lane-per-stream kernels with the slicer fused into the low-pass run: sps
    10 and sps 5), every stream's bytes and sync index == the oracle."""
    import _amr
    B, N = 8192, 96000
    x, want, wsync = _seeded_batch("qpsk", baud, B, N)
    plan = _amr.PskPlan("qpsk", N, baud, max_streams=B)
    plan.set_inflight(16)
    got, gsync = plan.demod_host(x)
    assert plan.last_layout() == "lane"
    mism = [i for i in range(B) if got[i] != want[i]]
    assert not mism, f"{len(mism)} streams differ, first {mism[:5]}"
    assert np.array_equal(gsync, wsync)


@pytest.mark.parametrize("layout", ["lane", "row"])
def test_ten_second_captures_past_2g_samples(layout):
    """10-s captures (960 000 samples, what decode_wav_file hands the demod
    after resampling a 10-s WAV, decoder.py:385-389) in a batch of 2304:
    2.2e9 samples, past 2^31, so every sample, state, checkpoint and symbol
    offset of both layouts must be 64-bit.  The batch cycles through 61
    distinct noisy captures (prime, so a stream that read another stream's
    rows, 64 or 128 groups away, would decode a different frame); every
    stream's bytes and sync index == the oracle's for its capture."""
    import _amr
    import synth
    from oracle import oracle
    B, N, U = 2304, 960000, 61
    assert B * N > 2 ** 31
    base = synth.qpsk_batch(U, N, 9600, seed=61, distinct=U)
    want, wsync = oracle.psk_demod_batch("qpsk", base, 9600, n_threads=min(16, os.cpu_count() or 1))
    x = base[np.arange(B) % U]
    plan = _amr.PskPlan("qpsk", N, 9600, max_streams=B)
    if layout == "lane":
        plan.set_inflight(16)
    got, gsync = plan.demod_host(x)
    assert plan.last_layout() == layout
    del plan
    mism = [i for i in range(B) if got[i] != want[i % U]]
    assert not mism, f"{len(mism)} streams differ, first {mism[:5]}"
    assert np.array_equal(gsync, wsync[np.arange(B) % U])


def test_ragged_streams():
    import modem
    from oracle import oracle
    rng = np.random.default_rng(5)
    streams = [rng.normal(0, 0.5, n).astype(np.float32) for n in (28, 100, 5000, 5000, 4999, 60)]
    got = modem.demodulate_ragged("qpsk", streams, 2400)
    for s, g in zip(streams, got):
        assert g == oracle.qpsk_demodulate(s, baud=2400)


def test_fec_gpu_matches_reference(golden):
    import fec
    manifest, _ = golden
    rs = fec.ReedSolomonFEC()
    ins = [bytes.fromhex(f["in"]) for f in manifest["fec"]]
    outs, oks = rs.decode_batch(ins)
    for f, o, ok, d in zip(manifest["fec"], outs, oks, ins):
        assert o.hex() == f["out"]
        if len(d) >= 4:
            assert ok == (not f["crc_warn"])
    buf = io.StringIO()
    with contextlib.redirect_stdout(buf):
        assert rs.decode(ins[-1]).hex() == manifest["fec"][-1]["out"]
    assert ("Aviso: CRC" in buf.getvalue()) == manifest["fec"][-1]["crc_warn"]


@pytest.mark.parametrize("B,layout", [(64, "row"), (64, "split"), (8192, "row"), (8192, "lane")])
def test_fec_fused_after_8psk_demod(B, layout):
    """Config 5: 8PSK@19200 demod + FEC decode fused on the device == oracle
    chain (psk_demod_batch then fec_decode, fec.py:34-69), every stream's
    demod bytes, sync index, FEC bytes and CRC flag -- at B=64 and at BASELINE
    configs[4]'s full batch of 8192, both as one batch alone (row layout) and
    as bench.py times it (16 in flight: lane layout, fused slicer at sps 5)."""
    import ctypes
    import _amr
    from oracle import oracle
    N = 96000
    x, dem, wsync = _seeded_batch("qpsk", 19200, B, N)
    plan = _amr.PskPlan("qpsk", N, 19200, max_streams=B)
    if layout == "lane":
        plan.set_inflight(16)
    elif B <= 64:
        plan.set_layout(layout)     # up to 64 streams the default is the time-split layout
    L = _amr.lib()
    cap = plan.out_cap
    ptrs = {}
    for name, nbytes in (("x", x.nbytes), ("out", B * cap), ("len", B * 8), ("sync", B * 8), ("fec", B * cap),
                         ("flen", B * 8), ("ok", B * 4)):
        p = ctypes.c_void_p()
        _amr.check(L.amr_malloc(ctypes.byref(p), nbytes))
        ptrs[name] = p
    host = {}
    try:
        _amr.check(L.amr_memcpy_h2d(ptrs["x"], _amr.ptr(x), x.nbytes))
        _amr.check(L.amr_psk_demod_fec_device(plan.handle, ptrs["x"], _amr.DTYPE_F32, B, N, ptrs["out"], cap,
                                              ptrs["len"], ptrs["sync"], ptrs["fec"], cap, ptrs["flen"], ptrs["ok"]))
        _amr.check(L.amr_psk_plan_synchronize(plan.handle))
        for name, shape, dt in (("out", (B, cap), np.uint8), ("len", B, np.int64), ("sync", B, np.int64),
                                ("fec", (B, cap), np.uint8), ("flen", B, np.int64), ("ok", B, np.int32)):
            host[name] = np.empty(shape, dt)
            _amr.check(L.amr_memcpy_d2h(_amr.ptr(host[name]), ptrs[name], host[name].nbytes))
    finally:
        for p in ptrs.values():
            L.amr_free(p)
    assert plan.last_layout() == layout
    assert np.array_equal(host["sync"], wsync)
    bad = []
    for i in range(B):
        want, wok = oracle.fec_decode(dem[i])
        if (host["out"][i, :host["len"][i]].tobytes() != dem[i] or host["fec"][i, :host["flen"][i]].tobytes() != want
                or bool(host["ok"][i]) != wok):
            bad.append(i)
    assert not bad, f"{len(bad)} of {B} streams differ, first {bad[:5]}"


def test_decode_wav_file_end_to_end(golden, tmp_path, monkeypatch):
    import decoder
    manifest, inputs = golden
    monkeypatch.chdir(tmp_path)
    for case in manifest["decoder"]:
        p = tmp_path / (case["id"] + ".wav")
        p.write_bytes(inputs[case["id"]].tobytes())
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            saved = decoder.decode_wav_file(str(p), case["mode"], case["symbol_rate"])
        got = []
        for s in saved:
            with open(s, "rb") as f:
                got.append({"name": os.path.basename(s).split("_", 1)[1], "data": f.read().hex()})
        assert got == case["files"], case["id"]


@pytest.mark.parametrize("layout", ["row", "split"])
def test_timing_hooks(layout):
    """Per-stage HIP-event times of a call; the time-split layout times its
    two low-pass passes in the lowpass_fwd slot and its gated serial fallback
    in lowpass_exact."""
    import _amr
    import synth
    x = synth.qpsk_batch(64, 20000, 9600, seed=1, distinct=2)
    plan = _amr.PskPlan("qpsk", 20000, 9600, max_streams=64)
    plan.set_layout(layout)
    plan.enable_timing(True)
    plan.demod_host(x)
    assert plan.last_layout() == layout
    t = plan.timings()
    want = {"bandpass", "lowpass_fwd", "lowpass_bwd", "sync_pack"} if layout == "row" else \
        {"bandpass", "lowpass_fwd", "lowpass_exact", "sync_pack"}
    assert set(t) >= want
    assert all(v > 0 for v in t.values())


def test_decode_wav_file_44k_qpsk_through_gpu_resample(tmp_path, monkeypatch):
    """A 44.1 kHz QPSK@1000 WAV: decode_wav_file (GPU resample + GPU demod) ==
    scipy.signal.resample + the oracle demod + the host frame parse, i.e. the
    reference's decode_wav_file pipeline (decoder.py:380-389) restated on the CPU.
    The GPU resample is scipy's bit for bit (test_gpu_fsk.py::test_resample_matches_scipy),
    and here equal to the oracle's pocketfft restatement (oracle.resample) and
    to scipy's on the recording itself; the decoded bytes and saved files are
    compared exactly (the reference's own decode_wav_file outputs at 44.1 / 48
    / 22.05 kHz are pinned by tests/test_gpu_wav.py)."""
    import decoder
    import synth
    from oracle import oracle
    from scipy import signal
    rng = np.random.default_rng(44)
    fr = synth.random_frame(rng, 300, name="wav44.bin")
    x = synth.qpsk_waveform(fr, 1000)                          # 96 kHz, as the reference transmits
    x = np.concatenate([np.zeros(4000, np.float32), x, np.zeros(6000, np.float32)])
    x = signal.resample(x.astype(np.float64), int(round(x.size * 44100 / 96000)))   # a 44.1 kHz recording
    x = 0.8 * x + rng.normal(0, 0.02, x.size)
    p = tmp_path / "q44.wav"
    p.write_bytes(synth.wav_bytes(np.clip(x, -1, 1), 44100))
    monkeypatch.chdir(tmp_path)
    with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
        saved = decoder.decode_wav_file(str(p), "QPSK", 1000)
    data, sr = decoder._read_wav(str(p))
    if data.dtype == np.int16:
        data = data.astype(np.float64) / 32768.0          # what libsndfile hands the reference (decoder.py:381)
    import _amr
    num = int(round(len(data) * 96000.0 / sr))
    y = signal.resample(data, num)
    assert np.array_equal(oracle.resample(data, num), y)
    assert np.array_equal(_amr.resample(data, num), y)
    raw = oracle.qpsk_demodulate(y, baud=1000)
    with contextlib.redirect_stdout(io.StringIO()):
        frames = decoder.parse_fbp_stream_enhanced(raw)
    assert [os.path.basename(s).split("_", 1)[1] for s in saved] == [f["name"] for f in frames]
    assert [f["name"] for f in frames] == ["wav44.bin"]
    import compression
    with open(saved[0], "rb") as f:
        assert f.read() == compression.intelligent_decompress(frames[0]["data"])


def test_group8_bandpass_forced_on_every_golden_case(tmp_path):
    """K1g (the 8-lane-group band-pass the library picks above 4 streams per
    SIMD) forced on for small batches: every golden PSK case, f64 and int16
    inputs and a ragged 33-stream batch, against the reference / the oracle.
    One subprocess (AMR_BP_G8 is read once per process)."""
    import os
    import subprocess
    import sys
    script = tmp_path / "g8.py"
    script.write_text(f'''
import sys
sys.path[:0] = [{os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "audio-modem-radio_amd")!r},
                {os.path.dirname(os.path.dirname(os.path.abspath(__file__)))!r},
                {os.path.dirname(os.path.abspath(__file__))!r}]
import json, numpy as np
import modem, synth
from oracle import oracle
from _util import call_case, expected, outcome
g = {os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")!r}
manifest = json.load(open(g + "/manifest.json"))
inputs = np.load(g + "/inputs.npz")
bad = [c["id"] for c in manifest["cases"] if not c["fn"].startswith("fsk")
       and outcome(lambda: call_case(modem, c, inputs[c["id"]])) != expected(c)]
x = synth.qpsk_batch(33, 20011, 9600, seed=4, distinct=5)
for dt in (np.float32, np.float64):
    got = modem.qpsk_demodulate_batch(x.astype(dt), baud=9600)
    want, _ = oracle.psk_demod_batch("qpsk", x.astype(dt), 9600)
    bad += [f"{{dt.__name__}}[{{i}}]" for i in range(33) if got[i] != want[i]]
pcm = (x * 20000).astype(np.int16)
got = modem.qpsk_demodulate_batch(pcm, baud=9600)
want, _ = oracle.psk_demod_batch("qpsk", pcm, 9600)
bad += [f"int16[{{i}}]" for i in range(33) if got[i] != want[i]]
xb = synth.qpsk_batch(9, 30000, 1200, seed=5, distinct=3)
got = modem.bpsk_demodulate_batch(xb, baud=1200)
want, _ = oracle.psk_demod_batch("bpsk", xb, 1200)
bad += [f"bpsk[{{i}}]" for i in range(9) if got[i] != want[i]]
print("BAD", bad)
sys.exit(1 if bad else 0)
''')
    env = dict(os.environ, AMR_BP_G8="1")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


def test_pcm16_wav_path_equals_float64_path():
    """decode_wav_file hands 16-bit 96 kHz WAV samples to the GPU as int16
    (pcm / 32768 converted on the device): the bytes equal the float64 path's
    (the reference's libsndfile reading) for PSK, BPSK and FSK."""
    import modem
    import synth
    rng = np.random.default_rng(77)
    for kind, baud in (("qpsk", 9600), ("qpsk", 1000), ("bpsk", 1200)):
        wave_ = synth.qpsk_batch(3, 30001, baud, seed=baud) if kind == "qpsk" else \
            np.stack([synth.fit(synth.bpsk_waveform(synth.random_frame(rng, 60), baud), 30001) for _ in range(3)])
        for x in wave_:
            pcm = np.clip(x * 32767 + rng.normal(0, 30, x.size), -32768, 32767).astype(np.int16)
            want = (modem.qpsk_demodulate if kind == "qpsk" else modem.bpsk_demodulate)(pcm / 32768.0, baud)
            assert modem._pcm16_psk(kind, pcm, baud) == want, (kind, baud)
    for x in synth.fsk_batch(3, 24000, 9600, seed=5):
        pcm = (x * 20000).astype(np.int16)
        want = modem.fsk_demodulate(pcm / 32768.0, 9600, 12000.0, 24000.0)
        assert modem._pcm16_fsk(pcm, 9600, 12000.0, 24000.0) == want


def test_fsk_decide_global_form_forced(tmp_path):
    """The FSK decide kernel's global-memory form (taken for streams whose
    compare bits exceed its LDS staging, e.g. 20-s captures) forced at every
    length: seeded batches == oracle.  One subprocess (the switch is read once)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    script = tmp_path / "fg.py"
    script.write_text(f'''
import sys
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import numpy as np
import _fsk, synth
from oracle import oracle
bad = []
for (B, N, baud, m, s) in ((24, 96000, 9600, 12000.0, 24000.0), (5, 30011, 4800, 8000.0, 16000.0)):
    x = synth.fsk_batch(B, N, baud, m, s, seed=B, distinct=4, noise=0.3)
    got, _ = _fsk.FskPlan(N, baud, m, s, max_streams=B).demod_host(x)
    bad += [(N, i) for i in range(B) if got[i] != oracle.fsk_demodulate(x[i], baud, m, s)]
print("BAD", bad)
sys.exit(1 if bad else 0)
''')
    env = dict(os.environ, AMR_FSK_DECIDE_GLOBAL="1")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=250)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("variant", ["default", "unfused", "lp_split", "bp_one_wave", "wpb1", "wpb2_no_zero_taps",
                                     "bp_prefwd", "bp_prefwd_no_zero_taps", "bp_ck2", "bp_ck2_no_zero_taps"])
def test_lane_layout_forced_on_every_case(tmp_path, variant):
    """The lane-per-stream kernels (psk_lane_kernels.hip: checkpointed
    band-pass and low-pass, picked when many streams are in flight) forced on
    for every call: every golden PSK case (incl. silence / -0.0 / denormal /
    NaN / inf streams through the detector and K3x), f64 and int16 inputs,
    BPSK, sps 5 / 10 / 20 and a generic sps, streams shorter than one tile,
    a ragged batch (B not a multiple of 64), streams that trip the band-pass
    zero-tap detector among ordinary ones, and the full 4096 x 96000 batch,
    against the reference / the oracle.  One subprocess per variant (the
    AMR_* switches are read once per process): the default kernels with the
    slicer fused into the low-pass forced on (AMR_FUSED_SLICE=1) and off, the
    role-split low-pass (AMR_LP_SPLIT=1), the one-wave band-pass
    (AMR_BP_SPLIT=0), one-wave / one-group workgroups (AMR_LANE_WPB=1), and
    2-wave workgroups with every band-pass tap computed (AMR_LANE_WPB=2,
    AMR_BP_ZO=0); the variants skip the full 4096-stream batch."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    script = tmp_path / "lane.py"
    script.write_text(f'''
import sys, os
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import json, numpy as np
import _amr, modem, synth
from oracle import oracle
from _util import call_case, expected, outcome
g = {os.path.join(here, "golden")!r}
manifest = json.load(open(g + "/manifest.json"))
inputs = np.load(g + "/inputs.npz")
bad = [c["id"] for c in manifest["cases"] if not c["fn"].startswith("fsk")
       and outcome(lambda: call_case(modem, c, inputs[c["id"]])) != expected(c)]
nt = min(16, os.cpu_count() or 1)
def check(kind, x, baud, tag):
    pl = _amr.PskPlan(kind, x.shape[1], baud, max_streams=x.shape[0])
    got, gs = pl.demod_host(x)
    assert pl.last_layout() == "lane", pl.last_layout()
    want, ws = oracle.psk_demod_batch(kind, x, baud, n_threads=nt)
    return [f"{{tag}}[{{i}}]" for i in range(x.shape[0]) if got[i] != want[i] or gs[i] != ws[i]]
x = synth.qpsk_batch(97, 20011, 9600, seed=4, distinct=7)
for dt in (np.float32, np.float64):
    bad += check("qpsk", x.astype(dt), 9600, dt.__name__)
bad += check("qpsk", (x * 20000).astype(np.int16), 9600, "int16")
bad += check("bpsk", synth.qpsk_batch(9, 30000, 1200, seed=5, distinct=3), 1200, "bpsk1200")
bad += check("bpsk", synth.qpsk_batch(70, 20000, 9600, seed=6, distinct=3), 9600, "bpsk9600")
bad += check("qpsk", synth.dpsk8_batch(65, 24000, 19200, seed=7, distinct=5), 19200, "psk8")
bad += check("qpsk", synth.qpsk_batch(33, 30001, 4800, seed=8, distinct=5), 4800, "sps20")
bad += check("qpsk", synth.qpsk_batch(17, 30001, 2400, seed=9, distinct=5), 2400, "sps40")
bad += check("qpsk", synth.qpsk_batch(5, 39, 9600, seed=10, distinct=5), 9600, "n39")
# band-pass zero-tap detector: leading silence, -0.0 runs, a late inf and a
# NaN inside groups of ordinary streams (their groups re-run with every tap)
x = synth.qpsk_batch(130, 20000, 9600, seed=11, distinct=9)
x[3, :5000] = 0.0
x[64, :777] = -0.0
x[65, 19999] = np.inf
x[129, 12345] = np.nan
x[100, 4000:4100] = 0.0
x[101] = 0.0
bad += check("qpsk", x, 9600, "bpzo")
if {variant!r} in ("default", "bp_ck2"):
    bad += check("qpsk", synth.qpsk_batch(4096, 96000, 9600, seed=4096, distinct=8), 9600, "b4096")
print("BAD", bad[:20], len(bad))
sys.exit(1 if bad else 0)
''')
    env = dict(os.environ, AMR_PSK_LANE="1")
    env.update({"default": {"AMR_FUSED_SLICE": "1"}, "unfused": {"AMR_FUSED_SLICE": "0"},
                "lp_split": {"AMR_LP_SPLIT": "1"},
                "bp_one_wave": {"AMR_BP_SPLIT": "0"}, "wpb1": {"AMR_LANE_WPB": "1"},
                "wpb2_no_zero_taps": {"AMR_LANE_WPB": "2", "AMR_BP_ZO": "0"},
                "bp_prefwd": {"AMR_BP_PREFWD": "1"},
                "bp_prefwd_no_zero_taps": {"AMR_BP_PREFWD": "1", "AMR_BP_ZO": "0"},
                "bp_ck2": {"AMR_BP_CK": "2"}, "bp_ck2_no_zero_taps": {"AMR_BP_CK": "2", "AMR_BP_ZO": "0"}}[variant])
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=280)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]


def test_async_host_entry_stream_of_batches():
    """amr_psk_demod_host_async / amr_fsk_demod_host_async on two plans in
    turn (uploads of one batch overlapping the other's demod), page-locked
    and pageable inputs, a pitched output: every batch == the oracle."""
    import _amr
    import _fsk
    import synth
    from oracle import oracle
    L = _amr.lib()
    B, N = 48, 24000
    xs = [synth.qpsk_batch(B, N, 9600, seed=40 + k, distinct=6) for k in range(4)]
    plans = [_amr.PskPlan("qpsk", N, 9600, max_streams=B) for _ in range(2)]
    cap = plans[0].out_cap
    outs = [(np.zeros((B, cap + 3), np.uint8), np.zeros(B, np.int64), np.zeros(B, np.int64)) for _ in range(4)]
    _amr.check(L.amr_host_register(_amr.ptr(xs[0]), xs[0].nbytes))
    try:
        for k in range(4):
            pl = plans[k % 2]
            if k >= 2:
                _amr.check(L.amr_psk_plan_synchronize(pl.handle))
            o, ln, sy = outs[k]
            _amr.check(L.amr_psk_demod_host_async(pl.handle, _amr.ptr(xs[k]), _amr.DTYPE_F32, B, N, _amr.ptr(o),
                                                  cap + 3, _amr.ptr(ln), _amr.ptr(sy)))
        for pl in plans:
            _amr.check(L.amr_psk_plan_synchronize(pl.handle))
    finally:
        L.amr_host_unregister(_amr.ptr(xs[0]))
    for k in range(4):
        want, wsync = oracle.psk_demod_batch("qpsk", xs[k], 9600)
        o, ln, sy = outs[k]
        assert [o[i, :ln[i]].tobytes() for i in range(B)] == want
        assert np.array_equal(sy, wsync)
    xf = synth.fsk_batch(8, N, 9600, 12000.0, 24000.0, seed=3, distinct=4, noise=0.2)
    pf = _fsk.FskPlan(N, 9600, 12000.0, 24000.0, max_streams=8)
    o = np.zeros((8, pf.out_cap), np.uint8)
    ln = np.zeros(8, np.int64)
    sy = np.zeros(8, np.int64)
    _amr.check(L.amr_fsk_demod_host_async(pf.handle, _amr.ptr(xf), _amr.DTYPE_F32, 8, N, _amr.ptr(o), pf.out_cap,
                                          _amr.ptr(ln), _amr.ptr(sy)))
    _amr.check(L.amr_fsk_plan_synchronize(pf.handle))
    assert [o[i, :ln[i]].tobytes() for i in range(8)] == [oracle.fsk_demodulate(r, 9600, 12000.0, 24000.0) for r in xf]


@pytest.mark.parametrize("layout", ["row", "lane"])
def test_batch_of_flagged_streams(layout):
    """Every stream of a 1030-stream batch is a gated capture -- a burst, then
    >= 66 000 samples of digital silence, over which the filters decay to
    exact zeros and denormals -- or all silence, so the low-pass detector
    flags all of them and the whole batch takes K3x, the exact complex
    low-pass (checkpointed, one workgroup per 64-stream group).  Bytes and
    sync == the oracle, in both layouts."""
    import time
    import _amr
    import synth
    from oracle import oracle
    B, N = 1030, 96000
    x = synth.qpsk_batch(B, N, 9600, seed=99, distinct=6)
    rng = np.random.default_rng(99)
    for i in range(B):
        x[i, 0 if i % 8 == 0 else int(rng.integers(8000, 30000)):] = 0.0
    plan = _amr.PskPlan("qpsk", N, 9600, max_streams=B)
    if layout == "lane":
        plan.set_inflight(16)
    plan.demod_host(x[:64])                                  # warm up (first-call allocations)
    t0 = time.perf_counter()
    got, gsync = plan.demod_host(x)
    dt = time.perf_counter() - t0
    assert plan.last_layout() == layout
    assert plan.exact_streams() == B
    want, wsync = oracle.psk_demod_batch("qpsk", x, 9600, n_threads=min(16, os.cpu_count() or 1))
    mism = [i for i in range(B) if got[i] != want[i]]
    assert not mism, f"{len(mism)} streams differ, first {mism[:5]}"
    assert np.array_equal(gsync, wsync)
    print(f"all-flagged {B} x {N} ({layout}): {dt * 1e3:.1f} ms host call")


def test_failed_scratch_grow_leaves_plan_usable(tmp_path):
    """The row layout grows a plan's s1 / s3 on its first call.  With every
    grow forced to fail (AMR_TEST_FAIL_SCRATCH_GROW=1): the row call raises
    AmrError (no memory) and the plan's lane-layout buffers are still intact,
    so the next lane call is == the oracle (no kernel ever sees freed memory)."""
    import subprocess
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    root = os.path.dirname(here)
    script = tmp_path / "grow.py"
    script.write_text(f'''
import sys
sys.path[:0] = [{os.path.join(root, "audio-modem-radio_amd")!r}, {root!r}, {here!r}]
import numpy as np
import _amr, synth
from oracle import oracle
x = synth.qpsk_batch(70, 24000, 9600, seed=3, distinct=5)
want, _ = oracle.psk_demod_batch("qpsk", x, 9600)
pl = _amr.PskPlan("qpsk", 24000, 9600, max_streams=70)
pl.set_inflight(1000)
assert pl.demod_host(x)[0] == want and pl.last_layout() == "lane"
before = pl.scratch_bytes()
pl.set_inflight(1)
try:
    pl.demod_host(x)
    raise SystemExit("row call did not fail")
except _amr.AmrError as e:
    assert e.code == _amr.AMR_E_NOMEM, e
pl.set_inflight(1000)
assert pl.demod_host(x)[0] == want and pl.last_layout() == "lane"
assert pl.scratch_bytes() == before, (pl.scratch_bytes(), before)
print("OK")
''')
    env = dict(os.environ, AMR_TEST_FAIL_SCRATCH_GROW="1")
    r = subprocess.run([sys.executable, str(script)], env=env, capture_output=True, text=True, timeout=200)
    assert r.returncode == 0 and "OK" in r.stdout, r.stdout[-2000:] + r.stderr[-2000:]


@pytest.mark.parametrize("first", [5, 20, 21, 55, 397])
def test_lane_layout_any_first(first):
    """The C ABI takes any first symbol index (amr_psk_plan_create); the
    reference's are sps // 2 and sps (modem.py:209, :92).  The lane kernels'
    static symbol slots hold only while first <= their tile; later ones take
    the generic path.  Bytes and sync == the oracle run with the same first."""
    import ctypes
    import _amr
    import synth
    from oracle import oracle
    B, N, baud = 70, 24000, 9600
    x = synth.qpsk_batch(B, N, baud, seed=first, distinct=5)
    sps, _, (b, a, zi), (bl, al, zil), lo4 = _amr.design_psk("qpsk", N, baud)
    h = ctypes.c_void_p()
    _amr.check(_amr.lib().amr_psk_plan_create(ctypes.byref(h), _amr.default_device(), _amr.PSK_QPSK, N, sps, first,
                                              _amr.ptr(b), _amr.ptr(a), _amr.ptr(zi), len(b), _amr.ptr(bl),
                                              _amr.ptr(al), _amr.ptr(zil), len(bl), _amr.ptr(lo4), B))
    try:
        _amr.check(_amr.lib().amr_psk_plan_set_inflight(h, 1000))
        cap = int(_amr.lib().amr_psk_plan_out_capacity(h))
        out = np.zeros((B, cap), np.uint8)
        ln = np.zeros(B, np.int64)
        sy = np.zeros(B, np.int64)
        _amr.check(_amr.lib().amr_psk_demod_host(h, _amr.ptr(x), _amr.DTYPE_F32, B, N, _amr.ptr(out), cap,
                                                 _amr.ptr(ln), _amr.ptr(sy)))
        assert _amr.lib().amr_psk_plan_last_layout(h) == 1
    finally:
        _amr.lib().amr_psk_plan_destroy(h)
    op = oracle.PskPlan("qpsk", N, baud)
    ocap = (2 * N) // sps // 8 + 8
    wout = np.zeros((B, ocap), np.uint8)
    wln = np.zeros(B, np.int64)
    wsy = np.zeros(B, np.int64)
    ob, oa, ozi = op.bp
    obl, oal, ozil = op.lp
    P = oracle._p
    oracle.lib().oracle_psk_demod_batch(0, P(x), oracle.DT_F32, B, N, N, sps, first, P(ob), P(oa), len(ob), P(ozi),
                                        P(obl), P(oal), len(obl), P(ozil), P(op.lo), P(wout), ocap, P(wln), P(wsy), 8)
    assert np.array_equal(ln, wln) and np.array_equal(sy, wsy)
    assert all(out[i, :ln[i]].tobytes() == wout[i, :wln[i]].tobytes() for i in range(B))
