import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU and the built HIP library")


def pytest_sessionstart(session):
    """Build provenance (moss_tts_amd/_buildid.py): a prebuilt libmtts.so or ASan driver whose
    compiled-in source hash is not this tree's fails the session before any test runs.  The ids are
    read from the binaries' bytes: nothing is loaded here (the HIP runtime must first come from
    torch's import, as in every test)."""
    from moss_tts_amd import _buildid
    for binary, scope in ((os.path.join(ROOT, "moss_tts_amd", "lib", "libmtts.so"), "lib"),
                          (os.path.join(ROOT, "tests", "native", "asan_driver"), "asan")):
        if not os.path.exists(binary):
            continue
        built, tree = _buildid.read_id(binary), _buildid.tree_hash(scope)
        if built != tree:
            pytest.exit(f"stale {binary}: built from sources {str(built)[:16]}, the tree's hash is {tree[:16]} "
                        "(rebuild: python -c 'import __graft_entry__ as g; g.build()')", returncode=3)


@pytest.fixture(scope="session")
def golden():
    import json
    import numpy as np
    d = os.path.join(ROOT, "tests", "golden")
    g = np.load(os.path.join(d, "golden.npz"), allow_pickle=False)
    with open(os.path.join(d, "cases.json")) as f:
        cases = json.load(f)
    return g, cases
