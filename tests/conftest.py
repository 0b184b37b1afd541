import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:  # test helpers (archive_util)
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def oracle_lib():
    from oracle import oracle as O
    O.build()
    return O


@pytest.fixture(scope="session")
def synth_small_path():
    from fishnet_amd import synthnet
    return synthnet.cached_synth_net(128, 2)


@pytest.fixture(scope="session")
def synth_big_path():
    from fishnet_amd import synthnet
    return synthnet.cached_synth_net(3072, 1)


@pytest.fixture(scope="session")
def oracle_nets(oracle_lib, synth_big_path, synth_small_path):
    return oracle_lib.Net(synth_big_path), oracle_lib.Net(synth_small_path)


@pytest.fixture(scope="session")
def gpu_ctx(synth_big_path, synth_small_path):
    from fishnet_amd import build, gpu_nnue
    build.build()
    return gpu_nnue.GpuNnue(synth_big_path, synth_small_path)
