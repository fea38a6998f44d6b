"""The product library's runtime knobs (csrc/dofs_knobs.h): dofs_create reads every DOFS_*
environment variable and refuses an unknown name or an invalid value, so a misspelt or retired knob can never
select a path silently. Runs on the host emulator's build of the same C-ABI (CPU); the GPU build shares the
code (dofs_cabi.inc.h)."""
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
EMU = os.path.join(ROOT, "tests", "emu", "_build", "libdofs_emu.so")


@pytest.fixture()
def emu_lib():
    from conftest import locked_make
    locked_make(os.path.join(ROOT, "tests", "emu"))
    return EMU


@pytest.mark.parametrize("name,value,why", [
    ("DOFS_REPLAY_FLOW", "0", "not a knob"),      # retired in round 5 (the round-launch replay is gone)
    ("DOFS_FUSED", "0", "not a knob"),
    ("DOFS_KEYFAST", "0", "not a knob"),          # a test entry now (dofs_debug_replay_keyfast)
    ("DOFS_SKIP_B", "1", "not a knob"),           # measurement builds only (-DDOFS_MEASURE)
    ("DOFS_B_DELAY", "1000", "not a knob"),       # measurement builds only
    ("DOFS_FLOW_LONG", "abc", "not a valid value"),
    ("DOFS_FLOW_LONG", "2", "not a valid value"),
    ("DOFS_FLOW_LONG", "100000", "not a valid value"),
    ("DOFS_SERIAL", "2", "not a valid value"),
    ("DOFS_KRT_DNC", "", "not a valid value"),
    ("DOFS_LONG_PATH", "8", "not a valid value"),
])
def test_create_refuses_unknown_or_invalid(monkeypatch, emu_lib, name, value, why):
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    monkeypatch.setenv(name, value)
    with pytest.raises(RuntimeError, match=f"{name}.*{why}"):
        Dofs(0, lib=emu_lib)


@pytest.mark.parametrize("env", [{"DOFS_SERIAL": "1"}, {"DOFS_FLOW_LONG": "256"}, {"DOFS_LONG_PATH": "64"},
                                 {"DOFS_KRT_DNC": "0"}, {"DOFS_PRE_JUMP": "0"}, {"DOFS_LIB": EMU}])
def test_create_accepts_the_knobs(monkeypatch, emu_lib, env):
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    Dofs(0, lib=emu_lib).close()


def test_only_the_listed_knobs_are_read():
    """Every getenv of the product sources is in dofs_knobs.h (the one place that validates them)."""
    import glob
    import re
    srcs = glob.glob(os.path.join(ROOT, "denseopticalflowsegmentation3d_amd", "csrc", "*.h")) + \
        glob.glob(os.path.join(ROOT, "denseopticalflowsegmentation3d_amd", "csrc", "*.hip"))
    for p in srcs:
        if os.path.basename(p) == "dofs_knobs.h":
            continue
        assert not re.search(r"\bgetenv\s*\(", open(p).read()), p
    names = set(re.findall(r'name == "(DOFS_[A-Z_0-9]+)"', open(os.path.join(
        ROOT, "denseopticalflowsegmentation3d_amd", "csrc", "dofs_knobs.h")).read()))
    assert names == {"DOFS_SERIAL", "DOFS_FLOW_LONG", "DOFS_LONG_PATH", "DOFS_KRT_DNC", "DOFS_PRE_JUMP",
                     "DOFS_LIB", "DOFS_SKIP_B", "DOFS_SKIPMASK", "DOFS_B_DELAY"}


def test_knobs_are_per_context(monkeypatch, emu_lib):
    """Each context keeps the knobs of the environment it was created in: a context created
    later under another DOFS_FLOW_LONG does not change an earlier one's."""
    from denseopticalflowsegmentation3d_amd.runtime import Dofs
    monkeypatch.setenv("DOFS_FLOW_LONG", "64")
    monkeypatch.setenv("DOFS_LONG_PATH", "128")
    a = Dofs(0, lib=emu_lib)
    monkeypatch.setenv("DOFS_FLOW_LONG", "512")
    monkeypatch.delenv("DOFS_LONG_PATH")
    b = Dofs(0, lib=emu_lib)
    try:
        assert a.knobs()["flow_long"] == 64 and a.knobs()["long_path"] == 128
        assert b.knobs()["flow_long"] == 512 and b.knobs()["long_path"] == 0
        monkeypatch.delenv("DOFS_FLOW_LONG")
        c = Dofs(0, lib=emu_lib)
        assert c.knobs()["flow_long"] == 0 and a.knobs()["flow_long"] == 64
        c.close()
    finally:
        a.close()
        b.close()


def test_create_error_is_per_thread(monkeypatch, emu_lib):
    """dofs_last_error(NULL) is the calling thread's last failed dofs_create: a create on another
    thread neither changes nor invalidates it, and creates on many threads at once do not race."""
    import ctypes as C
    import threading

    from denseopticalflowsegmentation3d_amd.runtime import Dofs, load
    lib = load(emu_lib)
    lib.dofs_create.restype = C.c_void_p
    lib.dofs_last_error.argtypes = [C.c_void_p]
    lib.dofs_last_error.restype = C.c_char_p
    monkeypatch.setenv("DOFS_SERIAL", "7")
    assert not lib.dofs_create(0)
    mine = lib.dofs_last_error(None).decode()
    assert "DOFS_SERIAL=7" in mine
    monkeypatch.delenv("DOFS_SERIAL")
    errs, others = [], []

    def worker():
        try:
            for _ in range(20):
                Dofs(0, lib=emu_lib).close()
            others.append(lib.dofs_last_error(None).decode())
        except Exception as e:  # pragma: no cover - reported below
            errs.append(e)

    ts = [threading.Thread(target=worker) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert others == ["null context"] * 4
    assert lib.dofs_last_error(None).decode() == mine
