"""The C-ABI library builds, loads without a GPU, and exports every symbol include/dofs.h declares."""
import ctypes
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols(header="dofs.h"):
    src = open(os.path.join(ROOT, "include", header)).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(dofs_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_entry_points():
    names = declared_symbols()
    for n in ("dofs_create", "dofs_segment", "dofs_segment_batch_device", "dofs_lift", "dofs_calib",
              "dofs_intersect", "dofs_destroy", "dofs_batch_fetch"):
        assert n in names


def test_library_exports_every_declared_symbol():
    from denseopticalflowsegmentation3d_amd import runtime
    lib = runtime.load()
    missing = [n for n in declared_symbols() if not hasattr(lib, n)]
    assert not missing, missing


def test_rccl_library_exports_every_declared_symbol():
    """libdofs_rccl.so (include/dofs_rccl.h) loads without a GPU and exports its entry points."""
    from denseopticalflowsegmentation3d_amd import runtime
    lib = runtime.load_rccl()
    names = [n for n in declared_symbols("dofs_rccl.h") if n not in declared_symbols("dofs.h")]
    assert "dofs_gather_records" in names and "dofs_comm_init" in names
    missing = [n for n in names if not hasattr(lib, n)]
    assert not missing, missing
    assert lib.dofs_records_block_bytes(96, 64) == 4 * 96 + 96 * 96 * 64


def test_abi_version_and_struct_layouts():
    from denseopticalflowsegmentation3d_amd import abi, runtime
    lib = runtime.load()
    assert lib.dofs_abi_version() == 3
    p = abi.DofsParams()
    lib.dofs_default_params(ctypes.byref(p))
    ref = abi.default_params()
    assert bytes(p) == bytes(ref)
    # sizes fixed by the header (natural alignment, x86-64 and gfx950 alike)
    assert ctypes.sizeof(abi.DofsSolution) == 160 and ctypes.sizeof(abi.DofsSnapshot) == 208
    assert ctypes.sizeof(abi.DofsEvent) == 56 and ctypes.sizeof(abi.DofsBoxRecord) == 96
    assert ctypes.sizeof(abi.DofsEdge) == 16


def test_no_device_fails_loudly():
    """Without a gfx950 device dofs_create returns NULL (no CPU fallback)."""
    import pytest
    import torch
    if torch.cuda.is_available():
        pytest.skip("device present")
    from denseopticalflowsegmentation3d_amd import runtime
    with pytest.raises(RuntimeError):
        runtime.Dofs(0)
