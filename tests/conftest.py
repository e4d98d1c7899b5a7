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


# GPU tests run cheapest first (under `-x` a failure then stops before the hour-long full-size
# legs, and the box's time goes to the parity checks): kernels on small worlds, then the device
# pipeline paths, then the one-rank shapes of configs[3] / configs[4], the full-size C3 last
_GPU_ORDER = ["test_gpu_align", "test_gpu_tails", "test_gpu_blat", "test_gpu_genome", "test_gpu_s5s6",
              "test_gpu_shard", "test_gpu_dist", "test_filter_model", "test_pipeline", "test_singlecell",
              "test_gpu_configs", "test_gpu_c3"]


def pytest_collection_modifyitems(config, items):
    def rank(item):
        if item.get_closest_marker("gpu") is None:
            return -1  # CPU tests keep their place, ahead of any GPU test
        mod = os.path.splitext(os.path.basename(str(item.fspath)))[0]
        return _GPU_ORDER.index(mod) if mod in _GPU_ORDER else len(_GPU_ORDER) // 2
    items[:] = sorted(items, key=rank)  # stable: the file order inside a rank
