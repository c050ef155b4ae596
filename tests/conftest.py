import json
import os
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(REPO, "tests", "golden")
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs the HIP engine)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def load_json(name):
    with open(os.path.join(GOLDEN, name)) as f:
        return json.load(f)


@pytest.fixture(scope="session")
def vectors():
    return load_json("ed25519_vectors.json")


@pytest.fixture(scope="session")
def txn_fixtures():
    return load_json("txn_fixtures.json")["txns"]


@pytest.fixture(scope="session")
def misc_vectors():
    return load_json("misc_vectors.json")


@pytest.fixture(scope="session")
def sha_vectors():
    return load_json("sha512_cavp.json")


@pytest.fixture(scope="session")
def quic_corpus():
    d = np.load(os.path.join(GOLDEN, "quic_txns.npz"))
    return d["arena"], d["txns"], d["codes"]


@pytest.fixture(scope="session")
def oracle():
    from oracle import oracle as orc
    orc.lib()
    return orc


@pytest.fixture(scope="module")
def engine():
    from firedancer_amd import VerifyEngine
    e = VerifyEngine(0, max_txn=1 << 17, max_sig=1 << 18, max_arena=1 << 26)
    yield e
    e.close()


@pytest.fixture(scope="module")
def engine_ref():
    from firedancer_amd import VerifyEngine
    e = VerifyEngine(0, max_txn=1 << 12, max_sig=1 << 13, max_arena=1 << 22, ref_mapping=True)
    yield e
    e.close()
