"""Known-answer loopbacks: at the rates where the reference's own
modulator and demodulator round-trip, a framed payload modulated on the GPU
(modem.modulate_batch, modem.py:28-65 / 138-186 / 270-295) and demodulated
on the GPU (modem.*_demodulate_batch, the benchmarked kernels) comes back
byte for byte through the frame parser (decoder.py:142-208, payload CRC32):
  * QPSK at 600 / 1000 / 1500 / 3000 Bd (carrier 3000 Hz: the phase advances
    by whole turns per symbol);
  * FSK at 300 Bd with the reference's default tones 1200 / 2200 Hz, and at
    1200 Bd with 2400 / 4800 Hz (both tones above the baud);
  * decode_wav_file end to end at QPSK / 8PSK / OFDM8 @ 1000 Bd (encoder ->
    WAV -> decoder, decoder.py:380-389 dispatch): the file is recovered.
Each batch also goes through both PSK kernel layouts (row: one batch alone;
lane: the plan told 16 batches are in flight)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def _frames(n, payload_len, seed):
    import synth
    rng = np.random.default_rng(seed)
    return [synth.random_frame(rng, int(payload_len), name=f"p{i}.bin") for i in range(n)]


def _payloads(raws):
    import decoder
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        sets = decoder.parse_fbp_stream_enhanced_batch(raws)
    return [[f["data"] for f in fs] for fs in sets]


def _want_payload(frame):
    import decoder
    import contextlib
    import io
    with contextlib.redirect_stdout(io.StringIO()):
        fs = decoder.parse_fbp_stream_enhanced(frame)
    assert len(fs) == 1
    return fs[0]["data"]


@pytest.mark.parametrize("baud", [600, 1000, 1500, 3000])
@pytest.mark.parametrize("layout", ["row", "lane", "split"])
def test_qpsk_loopback(baud, layout):
    import _amr
    import modem
    frames = _frames(24, max(8, baud // 40), seed=baud)
    x = modem.modulate_batch("qpsk", frames, baud)
    plan = _amr.PskPlan("qpsk", x.shape[1], baud, max_streams=x.shape[0])
    if layout == "lane":
        plan.set_inflight(1024)
    else:
        plan.set_layout(layout)
    raws, _ = plan.demod_host(x)
    assert plan.last_layout() == layout or (layout == "split" and plan.last_layout() == "row")
    got = _payloads(raws)
    for i, fr in enumerate(frames):
        assert got[i] == [_want_payload(fr)], (baud, layout, i)


@pytest.mark.parametrize("baud,mark,space", [(300, 1200.0, 2200.0), (1200, 2400.0, 4800.0)])
def test_fsk_loopback(baud, mark, space):
    import modem
    frames = _frames(12, max(8, baud // 40), seed=baud + 1)
    x = modem.modulate_batch("fsk", frames, baud, mark, space)
    raws = modem.fsk_demodulate_batch(x, baud=baud, mark_freq=mark, space_freq=space)
    got = _payloads(raws)
    for i, fr in enumerate(frames):
        assert got[i] == [_want_payload(fr)], (baud, i)


@pytest.mark.parametrize("mode", ["QPSK", "8PSK", "OFDM8"])
def test_decode_wav_file_recovers_the_file(tmp_path, monkeypatch, mode):
    import decoder
    import encoder
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(len(mode))
    src = tmp_path / "payload.bin"
    data = bytes(rng.integers(0, 256, 700, dtype=np.uint8))
    src.write_bytes(data)
    wav = encoder.encode_file(str(src), mode, True, 1000)
    assert wav and os.path.exists(wav)
    saved = decoder.decode_wav_file(wav, mode, 1000)
    assert len(saved) == 1, saved
    with open(saved[0], "rb") as f:
        assert f.read() == data
