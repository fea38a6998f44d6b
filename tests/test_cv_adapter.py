"""include/dofs_cv.hpp — the reference's OpenCV signatures (get_segmented_array, build_graph, segment_graph,
get_bottom_variants, get_mat, get_mat_upper, get_intersect) over the C-ABI — compiled with g++ -Wall -Werror
against a test double of the few cv:: types it uses (tests/cv_adapter/mock: OpenCV is absent here) and run.
CPU: the host-only entries on the reference's test vectors. GPU: the device entries (segmentation round trip
through build_graph + segment_graph, get_best_segments, the lifting KAT)."""
import os
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIBDIR = os.path.join(ROOT, "denseopticalflowsegmentation3d_amd", "_build")


def _build(tmp_path):
    exe = str(tmp_path / "test_cv_adapter")
    cmd = ["g++", "-std=c++17", "-Wall", "-Wextra", "-Werror", "-I", os.path.join(ROOT, "tests", "cv_adapter", "mock"),
           "-I", os.path.join(ROOT, "include"), os.path.join(ROOT, "tests", "cv_adapter", "test_cv_adapter.cpp"),
           "-L", LIBDIR, "-ldofs_hip", f"-Wl,-rpath,{LIBDIR}", "-Wl,-rpath-link,/opt/rocm/lib", "-o", exe]
    subprocess.run(cmd, check=True)
    return exe


def test_adapter_compiles_and_host_entries(tmp_path):
    r = subprocess.run([_build(tmp_path)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert "cv adapter ok" in r.stdout


@pytest.mark.gpu
def test_adapter_device_entries(tmp_path):
    r = subprocess.run([_build(tmp_path), "device"], capture_output=True, text=True, timeout=120)
    assert r.returncode == 0, r.stderr
    assert "cv adapter ok" in r.stdout
