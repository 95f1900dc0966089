"""The C ABI boundary, without a GPU: the library builds for gfx950, loads,
exports every symbol include/amr.h declares, and fails LOUDLY (no CPU
fallback) when no device is present."""
import ctypes
import os
import re
import subprocess

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_symbols():
    with open(os.path.join(ROOT, "include", "amr.h")) as f:
        txt = f.read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t|double|const char \*)\s*\*?\s*(amr_\w+)\(", txt, re.M)))


def test_header_and_binding_agree():
    import _amr
    assert header_symbols() == sorted(_amr.EXPORTS)


def test_library_exports_every_header_symbol(built_lib):
    out = subprocess.run(["nm", "-D", "--defined-only", built_lib], capture_output=True, text=True, check=True).stdout
    exported = set(re.findall(r" T (amr_\w+)$", out, re.M))
    missing = set(header_symbols()) - exported
    assert not missing, missing


def test_library_has_gfx950_code_object(built_lib):
    with open(built_lib, "rb") as f:
        blob = f.read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob


def test_library_loads_and_reports_version(built_lib):
    import _amr
    L = _amr.lib()
    assert L.amr_abi_version() == 5


def test_demod_fails_loudly_without_gpu(built_lib):
    import _amr
    import modem
    if _amr.device_count() > 0:
        pytest.skip("a GPU is visible; this test is for the CPU container")
    x = np.zeros(5000, np.float32)
    with pytest.raises(_amr.AmrError):
        modem.qpsk_demodulate(x, baud=9600)
    with pytest.raises(_amr.AmrError):
        modem.bpsk_demodulate(x, baud=1200)
    with pytest.raises(_amr.AmrError):
        modem.fsk_demodulate(x, baud=9600, mark_freq=12000.0, space_freq=24000.0)
    with pytest.raises(_amr.AmrError):
        _amr.hilbert(np.zeros((1, 64)))


def test_fsk_plan_create_argument_checks(built_lib):
    import _amr
    L = _amr.lib()
    h = ctypes.c_void_p()
    b = np.zeros(7)
    a = np.zeros(7); a[0] = 1
    args = [_amr.ptr(v) for v in (b, a, b, b, a, b)]
    assert L.amr_fsk_plan_create(ctypes.byref(h), 0, 1000, 10, *args, 9, 1) == _amr.AMR_E_INVALID   # taps
    assert L.amr_fsk_plan_create(ctypes.byref(h), 0, 1000, 0, *args, 7, 1) == _amr.AMR_E_INVALID    # sps
    assert L.amr_fsk_plan_create(ctypes.byref(h), 0, 21, 10, *args, 7, 1) == _amr.AMR_E_PADLEN
    assert b"padlen, which is 21" in L.amr_last_error()
    args[1] = _amr.ptr(np.zeros(7))
    assert L.amr_fsk_plan_create(ctypes.byref(h), 0, 1000, 10, *args, 7, 1) == _amr.AMR_E_INVALID   # a[0]


def test_plan_create_argument_checks(built_lib):
    import _amr
    L = _amr.lib()
    h = ctypes.c_void_p()
    b = np.zeros(9)
    rc = L.amr_psk_plan_create(ctypes.byref(h), 0, 0, 10, 10, 5, _amr.ptr(b), _amr.ptr(b), _amr.ptr(b), 9,
                               _amr.ptr(b), _amr.ptr(b), _amr.ptr(b), 5, _amr.ptr(np.zeros(40)), 1)
    assert rc == _amr.AMR_E_INVALID          # a[0] != 1
    a = np.zeros(9); a[0] = 1
    rc = L.amr_psk_plan_create(ctypes.byref(h), 0, 0, 10, 10, 5, _amr.ptr(b), _amr.ptr(a), _amr.ptr(b), 9,
                               _amr.ptr(b), _amr.ptr(a), _amr.ptr(b), 5, _amr.ptr(np.zeros(40)), 1)
    assert rc == _amr.AMR_E_PADLEN
    assert b"padlen, which is 27" in L.amr_last_error()


def test_error_contract_precedes_device(built_lib, golden):
    """scipy's ValueErrors come from host-side design, before any device work,
    with the reference's exact message."""
    import modem
    manifest, inputs = golden
    from _util import call_case
    for case in manifest["cases"]:
        if case["status"] != "err" or case["fn"].startswith("fsk"):
            continue
        with pytest.raises(ValueError) as ei:
            call_case(modem, case, inputs[case["id"]])
        assert str(ei.value) == case["emsg"], case["id"]


def test_fsk_error_contract(built_lib, golden):
    import modem
    manifest, inputs = golden
    from _util import call_case
    for case in manifest["cases"]:
        if case["status"] == "err" and case["fn"].startswith("fsk"):
            with pytest.raises(ValueError) as ei:
                call_case(modem, case, inputs[case["id"]])
            assert str(ei.value) == case["emsg"], case["id"]


def test_frame_parse_argument_checks(built_lib):
    """Bad arguments are refused before any device work (amr_frame_parse_*)."""
    import _amr
    L = _amr.lib()
    cnt = np.zeros(2, np.int32)
    lens = np.array([4, 4], np.int64)
    buf = np.zeros((2, 4), np.uint8)
    recs = np.zeros((2, 4), _amr.FRAME_REC)
    assert L.amr_frame_parse_host(None, 4, _amr.ptr(lens), 2, 4, _amr.ptr(cnt), recs.ctypes.data) == _amr.AMR_E_INVALID
    assert L.amr_frame_parse_host(_amr.ptr(buf), 4, _amr.ptr(lens), 2, 0, _amr.ptr(cnt), recs.ctypes.data) == _amr.AMR_E_INVALID
    assert L.amr_frame_parse_device(None, None, 4, None, 2, 4, None, None) == _amr.AMR_E_INVALID
    assert L.amr_frame_parse_host(None, 0, None, 0, 1, None, None) == _amr.AMR_OK          # empty batch
    with pytest.raises(_amr.AmrError):
        _amr.frame_parse([b"FBPC"])                                                         # no GPU here


def test_set_inflight_argument_checks(built_lib):
    import _amr
    L = _amr.lib()
    assert L.amr_psk_plan_set_inflight(None, 2) == _amr.AMR_E_INVALID
    assert b"plan is NULL" in L.amr_last_error()


def test_build_id_matches_sources(built_lib):
    """amr_build_id() is the content hash of the sources the library was built
    from; it must equal the hash of this tree's sources (no stale binary)."""
    import _amr
    import build
    assert _amr.lib().amr_build_id().decode() == build.source_hash()


def test_frame_parse_max_cands_bound(built_lib):
    """The kernel keeps at most AMR_FRAME_MAX_CANDS (256) records per stream:
    a larger max_cands is refused instead of leaving records unwritten."""
    import _amr
    L = _amr.lib()
    cnt = np.zeros(1, np.int32)
    lens = np.array([4], np.int64)
    buf = np.zeros((1, 4), np.uint8)
    recs = np.zeros((1, 257), _amr.FRAME_REC)
    assert L.amr_frame_parse_host(_amr.ptr(buf), 4, _amr.ptr(lens), 1, 257, _amr.ptr(cnt),
                                  recs.ctypes.data) == _amr.AMR_E_INVALID
    assert b"AMR_FRAME_MAX_CANDS" in L.amr_last_error()
    assert L.amr_frame_parse_device(None, None, 4, None, 1, 257, None, None) == _amr.AMR_E_INVALID


def test_plan_byte_estimates_on_the_host(built_lib):
    """amr_*_plan_bytes_estimate are host arithmetic (no GPU): what the drop-in
    plan cache reserves before creating a plan.  BASELINE configs[2]'s
    16384-stream FSK plan (live-column layout: 1.4 x n complex per stream,
    the dead columns' transform kept apart -- 0.6 x n complex, which also
    takes the host-staged input -- so z survives F2 for the exact path, 2 GiB
    of envelope slots, and the time-split F1's forward outputs for a call of
    up to 1024 streams, 1.6 GB) stays under 56 GB, inside the cache's 64 GB;
    the natural layout (sps 80 at 96000) needs 3 x n plus staging."""
    import _amr
    L = _amr.lib()
    fsk = L.amr_fsk_plan_bytes_estimate(96000, 10, 7, 16384)
    assert 40e9 < fsk <= 56e9, fsk
    assert L.amr_fsk_plan_bytes_estimate(96000, 80, 7, 16384) > 1.6 * fsk
    psk = [L.amr_psk_plan_bytes_estimate(_amr.PSK_QPSK, 96000, 10, 5, 9, 5, b) for b in (1, 64, 4096, 8192)]
    assert all(a < b for a, b in zip(psk, psk[1:])) and psk[2] < 20e9
    assert L.amr_psk_plan_bytes_estimate(_amr.PSK_QPSK, 96000, 0, 5, 9, 5, 64) < 0
    assert L.amr_fsk_plan_bytes_estimate(96000, 10, 7, 0) < 0
