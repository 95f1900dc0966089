"""decoder.py's file handling around the demodulator vs the reference's own
outputs (tests/golden/assembly*, made by tests/golden/make_assembly_golden.py):
FileAssembly part quality / duplicate handling / reassembly, save_decoded_files
(files written, stats), and -- on the GPU -- decode_with_retry (return value and
the demodulated_attempt_<k>.bin dumps, whose bytes are three GPU demodulations
at 1500, 1425 and 1496 Bd)."""
import glob
import json
import os

import numpy as np
import pytest

G = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


@pytest.fixture(scope="module")
def asm_golden():
    with open(os.path.join(G, "assembly_manifest.json")) as f:
        cases = {c["id"]: c for c in json.load(f)["cases"]}
    return cases, np.load(os.path.join(G, "assembly.npz"))


def test_signal_quality(asm_golden):
    import decoder
    cases, arr = asm_golden
    fa = decoder.FileAssembly("q.bin", 1, 0, 0)
    n = 0
    for cid, c in cases.items():
        if cid.startswith("quality."):
            assert fa.calculate_signal_quality(arr[cid].tobytes()) == c["value"], cid
            n += 1
    assert n >= 8


def test_assembly_sequences(asm_golden, capsys):
    import decoder
    cases, arr = asm_golden
    parts = [arr[f"parts.{i}"].tobytes() for i in range(3)]
    meta = cases["parts.meta"]
    for cid, c in cases.items():
        if not cid.startswith("assemble."):
            continue
        asm = decoder.AdvancedFileAssembly("f.bin", 3, meta["size"], meta["crc"])
        rets = [asm.add_part(i, parts[src], q) for i, src, q in c["seq"]]
        assert rets == c["add_part"], cid
        assert (asm.parts_quality, asm.received_parts, asm.get_progress(), asm.get_missing_parts(),
                asm.get_quality_report()) == (c["quality"], c["received"], c["progress"], c["missing"],
                                              c["report"]), cid
        if c["status"] == "ok":
            assert asm.assemble_file() == arr[cid + ".out"].tobytes(), cid
        else:
            with pytest.raises(ValueError) as ei:
                asm.assemble_file()
            assert str(ei.value) == c["emsg"], cid
        assert not asm.is_expired()


def test_save_decoded_files(asm_golden, tmp_path, monkeypatch, capsys):
    import decoder
    cases, arr = asm_golden
    c = cases["save"]
    monkeypatch.chdir(tmp_path)
    entries = [(e[0], arr[f"save.entry.{k}"].tobytes(), e[1], e[2], e[3], e[4], e[5])
               for k, e in enumerate(c["entries"])]
    before = dict(decoder.reception_stats)
    saved = decoder.save_decoded_files(entries)
    assert [os.path.basename(p).split("_", 2)[2] for p in saved] == c["saved_suffixes"]
    for k, p in enumerate(saved):
        with open(p, "rb") as f:
            assert f.read() == arr[f"save.out.{k}"].tobytes(), p
    assert {k: decoder.reception_stats[k] - before[k] for k in ("total_files", "total_bytes")} == c["stats_delta"]
    assert decoder.reception_stats["success_rate"] == c["success_rate"]
    assert not decoder.file_assemblies                  # the completed multi-part file was released


@pytest.mark.gpu
def test_gpu_decode_with_retry(asm_golden, tmp_path, monkeypatch, capsys):
    import decoder
    cases, arr = asm_golden
    monkeypatch.chdir(tmp_path)
    x = arr["retry.x"]
    for tag in ("qpsk", "psk8", "fsk", "fallback"):
        c = cases[f"retry.{tag}"]
        for f in glob.glob("demodulated_attempt_*.bin"):
            os.remove(f)
        assert decoder.decode_with_retry(x, c["mode"], c["symbol_rate"]) == c["value"], tag
        dumps = sorted(os.path.basename(f) for f in glob.glob("demodulated_attempt_*.bin"))
        assert dumps == c["dumps"], tag
        for d in dumps:
            with open(d, "rb") as f:
                assert f.read() == arr[f"retry.{tag}.{d}"].tobytes(), (tag, d)
