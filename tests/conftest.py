"""Test configuration: repo root on sys.path, the product package registered under its
importable name, the ``gpu`` marker, and the two native libraries (re)built by make."""
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)
import afpkg  # noqa: E402,F401

GOLDEN = os.path.join(ROOT, "tests", "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run on the GPU box with -m gpu)")


@pytest.fixture(scope="session", autouse=True)
def _native_builds():
    # make's dependency rules rebuild a library older than its sources (a stale .so shipped to
    # the GPU box would otherwise be tested); up to date, each call is a no-op
    subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    subprocess.run(["make", "-s", "-j8", "-C", os.path.join(ROOT, "anchored-fusion_amd", "csrc")], check=True)
    yield


@pytest.fixture(scope="session")
def anchor():
    from anchored_fusion_amd import io as afio
    return afio.anchor_sequence(os.path.join(GOLDEN, "target_gene.fasta"))


@pytest.fixture(scope="session")
def bundled_pairs():
    from anchored_fusion_amd import io as afio
    return afio.read_pairs(os.path.join(GOLDEN, "test_sample_1.fastq.gz"),
                           os.path.join(GOLDEN, "test_sample_2.fastq.gz"))
