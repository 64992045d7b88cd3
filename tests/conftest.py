import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TESTS = os.path.dirname(os.path.abspath(__file__))
for p in (ROOT, TESTS, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

GOLDEN = os.path.join(TESTS, "golden")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (HIP device); run with -m gpu")


# Tests that spawn child processes (torch.distributed.run) must run before anything in the pytest
# process initialises the GPU: they go first, whatever the collection order
# (tests/test_batch_shard_gpu.py asserts the precondition itself).
SPAWN_FIRST = ("test_batch_shard_gpu.py", "test_rowshard_gpu.py")


def pytest_collection_modifyitems(session, config, items):
    def rank(it):
        name = os.path.basename(str(it.fspath))
        return SPAWN_FIRST.index(name) if name in SPAWN_FIRST else len(SPAWN_FIRST)
    items.sort(key=rank)


@pytest.fixture(scope="session")
def golden_dir():
    return GOLDEN
