"""decode_wav_file (decoder.py:380-389) at capture rates other than 96 kHz,
through the drop-in decoder on the GPU -- the bit-exact resample
(scipy.signal.resample restated on pocketfft's transforms, csrc/pocketfft_dev.h)
then the PSK demod -- against the REFERENCE's own saved files
(tests/golden/make_wav_golden.py: 44.1 / 48 / 22.05 kHz WAVs of QPSK, 8PSK
and OFDM8 @ 1000, QPSK @ 9600 and BPSK @ 1200 with digital-silence padding)."""
import contextlib
import io
import os

import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def gpu(built_lib):
    import _amr
    if _amr.device_count() < 1:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X")


def test_decode_wav_file_matches_reference_at_44k_48k(wav_golden, tmp_path, monkeypatch):
    import decoder
    manifest, wavs = wav_golden
    monkeypatch.chdir(tmp_path)
    for case in manifest["cases"]:
        p = tmp_path / (case["id"] + ".wav")
        p.write_bytes(wavs[case["id"]].tobytes())
        with contextlib.redirect_stdout(io.StringIO()), contextlib.redirect_stderr(io.StringIO()):
            saved = decoder.decode_wav_file(str(p), case["mode"], case["symbol_rate"])
        got = []
        for s in saved:
            with open(s, "rb") as f:
                got.append({"name": os.path.basename(s).split("_", 1)[1], "data": f.read().hex()})
        assert got == case["files"], case["id"]
