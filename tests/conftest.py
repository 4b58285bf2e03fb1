import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

GOLDEN = os.path.join(ROOT, "tests", "golden")
TEST1 = os.path.join(GOLDEN, "ERR2755197_test_1.fq")
TEST2 = os.path.join(GOLDEN, "ERR2755197_test_2.fq")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")


@pytest.fixture(scope="session")
def test_pair():
    with open(TEST1, "rb") as f1, open(TEST2, "rb") as f2:
        return f1.read(), f2.read()
