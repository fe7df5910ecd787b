import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, 'tests', 'golden')
if REPO not in sys.path:
    sys.path.insert(0, REPO)


def pytest_configure(config):
    config.addinivalue_line('markers', 'gpu: needs a gfx950 (MI355X) GPU and the built HIP library')


def golden(name):
    return np.load(os.path.join(GOLDEN, name + '.npz'), allow_pickle=False)


@pytest.fixture(scope='session')
def ctx():
    """Native context on cuda:0. No skip: a -m gpu run without a GPU must fail loudly."""
    from acinoset_amd import _native
    return _native.Context(int(os.environ.get('ACINOSET_DEVICE', 0)))
