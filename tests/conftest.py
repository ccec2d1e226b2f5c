import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "orb-ygz-slam_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (HIP device); runs on the GPU box")


def gpu_available():
    try:
        import ygzfe
        return ygzfe.device_count() > 0
    except Exception:
        return False


def _segv_trace():
    """YGZFE_SEGV_TRACE=path/to/libsegv_trace.so (tools/segv): native backtrace on a segfault."""
    path = os.environ.get("YGZFE_SEGV_TRACE")
    if path:
        import ctypes
        ctypes.CDLL(path).segv_trace_install()


@pytest.fixture(autouse=True)
def _segv_trace_each():
    _segv_trace()  # re-installed per test: a runtime may have replaced the handler
    yield


@pytest.fixture(scope="session")
def gpu():
    import ygzfe
    n = ygzfe.device_count()
    if n <= 0:
        pytest.fail("no HIP device visible: -m gpu tests must run on the GPU box (no CPU fallback exists)")
    return ygzfe


# headline-path parity first, so a -x stop reports the §8a rows before the §8f ones
_ORDER = ["test_gpu_extract.py", "test_gpu_extract_split.py", "test_gpu_align.py", "test_gpu_align_batch.py",
          "test_gpu_match.py", "test_gpu_match_search.py", "test_gpu_dropin.py", "test_gpu_compat.py"]


def pytest_collection_modifyitems(session, config, items):
    def rank(item):
        name = os.path.basename(str(item.fspath))
        return _ORDER.index(name) if name in _ORDER else len(_ORDER)
    items.sort(key=rank)  # stable: file-internal order kept
