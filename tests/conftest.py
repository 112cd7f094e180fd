"""Test configuration: `gpu` marker, repo root on sys.path, golden fixtures."""
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a HIP device (MI355X); run with -m gpu")


@pytest.fixture(scope="session")
def golden():
    with open(os.path.join(GOLDEN, "golden.json")) as f:
        return json.load(f)


def read_golden(rel):
    with open(os.path.join(GOLDEN, rel), "rb") as f:
        return f.read()


@pytest.fixture(scope="session")
def golden_inputs(golden):
    return {k: read_golden(v["file"]) for k, v in golden["inputs"].items()}


@pytest.fixture(scope="session")
def decode_blob():
    return read_golden("decode_blocks.bin")
