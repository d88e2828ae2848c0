import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) GPU")
    config.addinivalue_line("markers", "explib: compares kernel variants that only the experiments build "
                            "(build/libstem_kernel_amd_exp.so, sk_experiments() = 1) selects; run by "
                            "tests/test_explib.py in a child process on that library")


def _experiments_build():
    try:
        from stem_kernel_amd._lib import lib
        return lib().sk_experiments() == 1
    except Exception:  # noqa: BLE001 (no library: the tests fail on their own)
        return False


def pytest_collection_modifyitems(config, items):
    if not any("explib" in it.keywords for it in items) or _experiments_build():
        return
    skip = pytest.mark.skip(reason="kernel-variant switch: runs in tests/test_explib.py on the experiments build")
    for it in items:
        if "explib" in it.keywords:
            it.add_marker(skip)


@pytest.fixture(scope="session")
def gpu_ctx():
    import stem_kernel_amd as ska
    ctx = ska.Context(0)
    yield ctx
    ctx.close()
