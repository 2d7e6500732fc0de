import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")


@pytest.fixture(scope="session", autouse=True)
def built_libs():
    """Build the engine and oracle libraries once if they are missing."""
    lib = os.path.join(ROOT, "redrock_old_amd", "librr_serdes.so")
    olib = os.path.join(ROOT, "oracle", "librr_oracle.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-j8", "-C", os.path.join(ROOT, "redrock_old_amd", "csrc")], check=True)
    if not os.path.exists(olib):
        subprocess.run(["make", "-C", os.path.join(ROOT, "oracle")], check=True)
    yield


@pytest.fixture(scope="session")
def engine():
    """The batch pipeline (count + decode windows, the four encode kernels) for every batch size:
    RR_CTX_NO_SMALL, so small test batches still exercise the walks.  The one-launch kernels
    small batches take by default are tested through `engine_small` (tests/test_gpu_small.py)."""
    import redrock_old_amd as rr
    eng = rr.Engine(0)
    eng.set_options(rr.CTX_NO_SMALL)
    yield eng
    eng.close()


@pytest.fixture(scope="session")
def engine_small():
    """A context with the default options: batches of at most 4096 values in at most 128 KiB
    take the one-launch kernels."""
    import redrock_old_amd as rr
    eng = rr.Engine(0)
    yield eng
    eng.close()
