import os
import sys

import pytest

sys.path.insert(0, os.path.abspath(os.path.join(os.path.dirname(__file__), "..")))

# Per-xdist-worker thread budget (the reference's conftest does the same,
# ``sklearn/conftest.py:117-134``): N workers x all-core OpenMP / BLAS pools
# oversubscribe the host and spinning OpenMP barriers then crawl.  Set before
# any native library (host OpenMP, BLAS, torch) initialises its pool.
_workers = os.environ.get("PYTEST_XDIST_WORKER_COUNT")
if _workers:
    _per = str(max(1, (os.cpu_count() or 1) // int(_workers)))
    for _var in ("OMP_NUM_THREADS", "OPENBLAS_NUM_THREADS", "MKL_NUM_THREADS"):
        os.environ[_var] = _per
    try:
        import torch as _torch
        _torch.set_num_threads(int(_per))
    except Exception:  # pragma: no cover
        pass


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: test needs a real MI355X (HIP device)")
    config.addinivalue_line("markers", "slow: long-running test")


@pytest.fixture(scope="session")
def cuda():
    import torch
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    return torch.device("cuda", 0)
