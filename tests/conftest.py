import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a gfx950 (MI355X) device and the HIP library")


@pytest.fixture(scope="session")
def calib():
    from oracle import binding as ob
    return ob.calib()


@pytest.fixture(scope="session")
def gpu():
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    ctx = Dofs(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def emu():
    """Sequential host model of the product pipeline (tests/emu, test infrastructure only)."""
    import subprocess
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    here = os.path.join(ROOT, "tests", "emu")
    subprocess.run(["make", "-s", "-C", here], check=True)
    ctx = Dofs(0, lib=os.path.join(here, "_build", "libdofs_emu.so"))
    yield ctx
    ctx.close()
