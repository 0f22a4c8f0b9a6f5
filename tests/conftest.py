import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
for p in (os.path.join(ROOT, "hadoop-bam_amd"), os.path.join(ROOT, "oracle"), ROOT):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu on the GPU box)")


@pytest.fixture(scope="session")
def golden():
    return json.load(open(os.path.join(GOLDEN, "golden.json")))


@pytest.fixture(scope="session")
def test_bam():
    return open(os.path.join(GOLDEN, "test.bam"), "rb").read()


def golden_path(name):
    return os.path.join(GOLDEN, name)
