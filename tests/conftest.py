import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def locked_make(directory):
    """`make -s -C directory` under an exclusive file lock, so pytest-xdist workers that build
    the same test library at once do not load a half-written .so."""
    import fcntl
    import subprocess
    with open(os.path.join(directory, ".make.lock"), "w") as lk:
        fcntl.flock(lk, fcntl.LOCK_EX)
        subprocess.run(["make", "-s", "-C", directory], check=True)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and the HIP library")


@pytest.fixture(scope="session")
def calib():
    from oracle import binding as ob
    return ob.calib()


@pytest.fixture(scope="session")
def gpu():
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    ctx = Dofs(0, keep_events=True)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def emu():
    """Sequential host model of the product pipeline (tests/emu, test infrastructure only)."""
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    here = os.path.join(ROOT, "tests", "emu")
    locked_make(here)
    ctx = Dofs(0, lib=os.path.join(here, "_build", "libdofs_emu.so"), keep_events=True)
    yield ctx
    ctx.close()
