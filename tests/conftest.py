import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if REPO not in sys.path:
    sys.path.insert(0, REPO)
TESTS = os.path.dirname(os.path.abspath(__file__))
if TESTS not in sys.path:
    sys.path.insert(0, TESTS)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (runs through the HIP C-ABI)")
    config.addinivalue_line("markers", "slow: long CPU test")


class _Opts:
    """The library's process-default options (rt_set_default_options) for one test: set(**fields)
    changes them (fields of rt_options, diag bits by name), clear(*names) returns those fields to
    the library defaults; the previous defaults come back at teardown."""

    def __init__(self, rt):
        self.rt = rt
        self.saved = rt.default_options()

    def set(self, **fields):
        self.rt.set_default_options(self.rt.options(self.rt.default_options(), **fields))

    def clear(self, *names):
        base = self.rt.options()
        self.set(**{n: (bool(base.diag & self.rt.abi.RT_DIAG[n]) if n in self.rt.abi.RT_DIAG else getattr(base, n))
                    for n in names})

    def restore(self):
        self.rt.set_default_options(self.saved)


@pytest.fixture
def opts():
    import raytracinginoneweekend_amd as rt
    o = _Opts(rt)
    yield o
    o.restore()
