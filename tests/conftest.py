import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through libdccrgx.so on the GPU)")


import pytest  # noqa: E402


@pytest.fixture
def lib_options():
    """set(name, value): a libdccrgx test option (dccrgx_test_option) for this
    test only; every option set is returned to its default afterwards."""
    from dccrg_amd.grid import set_test_option
    names = []

    def set_(name, value):
        set_test_option(name, value)
        names.append(name)

    yield set_
    for n in names:
        set_test_option(n, None)
