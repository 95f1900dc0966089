import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "audio-modem-radio_amd")
for p in (PKG, ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (run with -m gpu)")


@pytest.fixture(scope="session")
def golden():
    import json

    import numpy as np
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "manifest.json")) as f:
        manifest = json.load(f)
    inputs = np.load(os.path.join(g, "inputs.npz"))
    return manifest, inputs


@pytest.fixture(scope="session")
def sweep_golden():
    """The reference's outputs over a seeded draw of configurations
    (tests/golden/make_sweep_golden.py)."""
    import json

    import numpy as np
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "sweep_manifest.json")) as f:
        manifest = json.load(f)
    return manifest, np.load(os.path.join(g, "sweep.npz"))


@pytest.fixture(scope="session")
def rawint_golden():
    """The reference's outputs on raw integer / bool / float16 captures, whose
    odd extension scipy forms in the array's dtype (tests/golden/make_rawint_golden.py)."""
    import json

    import numpy as np
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "rawint_manifest.json")) as f:
        manifest = json.load(f)
    return manifest, np.load(os.path.join(g, "rawint.npz"))


@pytest.fixture(scope="session")
def wav_golden():
    """The reference's decode_wav_file on 44.1 / 48 / 22.05 kHz WAVs
    (tests/golden/make_wav_golden.py)."""
    import json

    import numpy as np
    g = os.path.join(ROOT, "tests", "golden")
    with open(os.path.join(g, "wav_manifest.json")) as f:
        manifest = json.load(f)
    return manifest, np.load(os.path.join(g, "wav.npz"))


@pytest.fixture(scope="session")
def built_lib():
    """libamr.so, built in-tree if missing (hipcc cross-compiles without a GPU)."""
    import build
    return build.build()
