"""encoder.py / compression drop-in vs the reference's own outputs
(tests/golden/encoder*.{npz,json}, made by tests/golden/make_encoder_golden.py).

CPU: compression analysis, every compressor, framing, stats, file splitting and
audio validation, byte for byte.  GPU (-m gpu): encode_file / encode_file_parts
write the reference's WAV files byte for byte (their samples come from the
tx kernels), encode_files_batch equals encode_file per file, and
encode_file -> decode_wav_file recovers the original files."""
import json
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def enc_golden():
    with open(os.path.join(G, "encoder_manifest.json")) as f:
        cases = json.load(f)["cases"]
    return cases, np.load(os.path.join(G, "encoder.npz"))


def _cases(cases, *fns):
    out = [c for c in cases if c["fn"] in fns]
    assert out, fns
    return out


def _fn(name):
    import compression
    import encoder
    ic = compression.IntelligentCompressor()
    return {
        "IntelligentCompressor.analyze_data_pattern": ic.analyze_data_pattern,
        "intelligent_compress": compression.intelligent_compress,
        "intelligent_decompress": compression.intelligent_decompress,
        "super_compress": compression.super_compress,
        "compress_data": compression.compress_data,
        "compression.adaptive_compress": compression.adaptive_compress,
        "encoder.adaptive_compress": encoder.adaptive_compress,
        "calculate_transmission_stats": encoder.calculate_transmission_stats,
    }[name]


def test_compression_matches_reference(enc_golden):
    cases, arr = enc_golden
    n = 0
    for c in _cases(cases, "IntelligentCompressor.analyze_data_pattern", "intelligent_compress",
                    "intelligent_decompress", "super_compress", "compress_data",
                    "compression.adaptive_compress", "encoder.adaptive_compress"):
        data = arr[c["id"] + ".in"].tobytes()
        got = _fn(c["fn"])(data, *c["args"], **c["kw"])
        assert c["status"] == "ok", c
        if c["kind"] == "bytes":
            assert bytes(got) == arr[c["id"] + ".out"].tobytes(), c["id"]
        else:
            assert got == c["value"], c["id"]
        n += 1
    assert n > 250


def test_compress_decompress_round_trip(enc_golden):
    """intelligent_compress -> intelligent_decompress is the identity except the
    reference's RAW off-by-one (utils/compression.py:77 vs :114)."""
    import compression
    cases, arr = enc_golden
    for c in _cases(cases, "intelligent_compress"):
        data = arr[c["id"] + ".in"].tobytes()
        packed = compression.intelligent_compress(data, *c["args"], **c["kw"])
        back = compression.intelligent_decompress(packed)
        assert back == (data[1:] if packed.startswith(b"RAW") else data), c["id"]
        assert compression.super_decompress(compression.super_compress(data)) == (
            data[1:] if len(data) < 500 else data)


def test_framing_stats_split_verify(enc_golden, tmp_path):
    import encoder
    cases, arr = enc_golden
    for c in _cases(cases, "_frame_data"):
        i = int(c["id"].split(".")[1])
        fname, part, total = [("a.txt", 0, 1), ("photo.jpg", 2, 5), ("n" * 300, 0, 1), ("ção ünï.bin", 1, 2)][i]
        got = encoder._frame_data(fname, arr[c["id"] + ".in"].tobytes(), part, total, 123456 + i, 0xDEADBEEF - i)
        assert got == arr[c["id"] + ".out"].tobytes(), c["id"]
    for c in _cases(cases, "calculate_transmission_stats"):
        assert encoder.calculate_transmission_stats(*c["args"]) == c["value"], c["id"]
    for key in arr.files:
        if key.startswith("file."):
            (tmp_path / key[5:]).write_bytes(arr[key].tobytes())
    for c in _cases(cases, "split_file_for_transmission"):
        name, mode, sr, dur = c["id"][len("split."):].rsplit(".", 3)
        parts = encoder.split_file_for_transmission(str(tmp_path / name), mode, int(sr), int(dur))
        assert [[p[0], p[1].hex(), p[2], p[3], p[4], p[5]] for p in parts] == c["value"], c["id"]
    for c in _cases(cases, "get_encoding_stats"):
        name = c["args"][0]
        assert encoder.get_encoding_stats(str(tmp_path / name), *c["args"][1:]) == c["value"]
    for c in _cases(cases, "verify_audio_output"):
        assert encoder.verify_audio_output(arr[c["id"] + ".in"]) == c["value"], c["id"]


def test_encoder_surface():
    """The names filebeep_advanced_v2.py:23 imports, and the reference's others."""
    import encoder
    for name in ("encode_file", "cancel_encoding", "get_encoding_stats", "reset_encoding_cancel",
                 "clear_encoding_cache", "get_file_signature", "encode_file_parts",
                 "split_file_for_transmission", "calculate_transmission_stats", "_frame_data",
                 "verify_audio_output", "adaptive_compress", "encode_hellschreiber_text"):
        assert callable(getattr(encoder, name)), name
    encoder.cancel_encoding()
    assert encoder._encoding_cancelled
    encoder.reset_encoding_cancel()
    assert not encoder._encoding_cancelled


# ----------------------------------------------------------------------------- GPU
def _write_files(arr, d):
    for key in arr.files:
        if key.startswith("file."):
            (d / key[5:]).write_bytes(arr[key].tobytes())


@pytest.mark.gpu
def test_gpu_encode_file_wavs_match_reference(enc_golden, tmp_path, monkeypatch):
    import encoder
    cases, arr = enc_golden
    _write_files(arr, tmp_path)
    monkeypatch.chdir(tmp_path)
    for c in _cases(cases, "encode_file"):
        name, mode, comp, sr = c["args"]
        out = encoder.encode_file(str(tmp_path / name), mode, comp, sr)
        assert os.path.relpath(out, tmp_path) == c["path"]
        with open(out, "rb") as f:
            assert f.read() == arr[c["id"] + ".out"].tobytes(), c["id"]
    parts = [("p.bin", arr["parts.in"].tobytes(), 0, 1, 30, 7)]
    for c in _cases(cases, "encode_file_parts"):
        mode, comp, sr = c["args"]
        if c["status"] == "err":
            with pytest.raises(Exception) as ei:
                encoder.encode_file_parts(parts, mode, comp, sr)
            assert (type(ei.value).__name__, str(ei.value)) == (c["etype"], c["emsg"]), c["id"]
            continue
        outs = encoder.encode_file_parts(parts, mode, comp, sr)
        assert os.path.relpath(outs[0], tmp_path) == c["path"]
        with open(outs[0], "rb") as f:
            assert f.read() == arr[c["id"] + ".out"].tobytes(), c["id"]


@pytest.mark.gpu
def test_gpu_encode_files_batch_and_round_trip(enc_golden, tmp_path, monkeypatch):
    import decoder
    import encoder
    _, arr = enc_golden
    _write_files(arr, tmp_path)
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(5)
    names = []
    for i in range(12):
        p = tmp_path / f"f{i}.bin"
        p.write_bytes(rng.integers(0, 256, int(rng.integers(10, 900)), dtype=np.uint8).tobytes())
        names.append(str(p))
    for mode, sr in (("QPSK", 9600), ("BPSK", 4800), ("FSK9600", 9600)):
        outs = encoder.encode_files_batch(names, mode, True, sr)
        for p, o in zip(names, outs):
            with open(o, "rb") as f:
                batched = f.read()
            single = encoder.encode_file(p, mode, True, sr)
            with open(single, "rb") as f:
                assert f.read() == batched, (p, mode)
    # encode -> decode recovers the file at a rate where the reference's own
    # modulator and demodulator loop back (3000/baud an integer: the carrier phase
    # advances by whole turns per symbol; at 9600 Bd it advances 112.5 deg per
    # symbol and the reference's differential slicer misreads clean audio);
    # decode_wav_file saves under ./recv as "<timestamp>_<name>"
    for p in names[:4] + [str(tmp_path / "mid.txt")]:
        wav = encoder.encode_file(p, "QPSK", True, 1500)
        saved = decoder.decode_wav_file(wav, "QPSK", 1500)
        assert len(saved) == 1, (p, saved)
        with open(saved[0], "rb") as f, open(p, "rb") as g:
            got, want = f.read(), g.read()
        # intelligent_compress tags small files RAW, which decode strips one byte too
        # many of (the reference's off-by-one, kept): then the payload loses byte 0
        assert got == want or (len(want) < 200 and got == want[1:]), p


@pytest.mark.gpu
def test_gpu_batched_encode_decode_round_trip(tmp_path, monkeypatch):
    """The whole batched path end to end: 64 files -> intelligent_compress + FBPC
    frames -> one batched GPU modulation (QPSK@1500, a loop-back rate of the
    reference's modem) -> one batched GPU demodulation + frame parse
    (decode_from_buffer_batch) -> every file back, byte for byte (files under
    200 B lose byte 0 to the reference's RAW-tag off-by-one, kept)."""
    import compression
    import decoder
    import encoder
    import modem
    monkeypatch.chdir(tmp_path)
    rng = np.random.default_rng(11)
    files, frames = [], []
    for i in range(64):
        n = int(rng.integers(20, 600))
        data = (rng.integers(0, 256, n, dtype=np.uint8).tobytes() if i % 2
                else bytes(rng.choice(list(b"abcdef ghij\n"), n).astype(np.uint8)))
        files.append(data)
        frames.append(encoder._frame_data(f"f{i}.bin", compression.intelligent_compress(data), 0, 1, n,
                                          binascii_crc(data)))
    x = modem.modulate_batch("qpsk", frames, 1500)
    saved = decoder.decode_from_buffer_batch(x, "QPSK", 1500)
    assert len(saved) == 64
    for i, paths in enumerate(saved):
        assert len(paths) == 1, (i, paths)
        with open(paths[0], "rb") as f:
            got = f.read()
        want = files[i]
        assert got == (want[1:] if len(want) < 200 else want), i


def binascii_crc(data: bytes) -> int:
    import binascii
    return binascii.crc32(data) & 0xffffffff
