import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "voxtral.c_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
GOLDEN = os.path.join(ROOT, "tests", "golden")
sys.path.insert(0, GOLDEN)  # fixture builders (gen_*.py) are importable; their main() is not run


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libvoxtral_hip.so)")
    config.addinivalue_line("markers", "slow: full-size Voxtral-4B shapes (minutes)")
    config.addinivalue_line("markers", "cpu: runs without a GPU")


@pytest.fixture(scope="session")
def tiny_cfg():
    from vox_weights import TINY
    return TINY


@pytest.fixture(scope="session")
def tiny_weights(tiny_cfg):
    from vox_weights import synth_weights
    return synth_weights(tiny_cfg, seed=1)


@pytest.fixture(scope="session")
def jfk_samples():
    # samples/jfk.wav of the reference (11.0 s, 16 kHz mono s16), kept as a fixture
    import vox_oracle
    return vox_oracle.read_wav(os.path.join(GOLDEN, "jfk.wav"))
