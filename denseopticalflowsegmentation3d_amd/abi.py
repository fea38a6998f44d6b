"""ctypes mirrors of the C-ABI structs declared in include/dofs.h (layout must match exactly)."""
from __future__ import annotations

import ctypes as C

import numpy as np


class _NpMixin:
    @classmethod
    def np_dtype(cls) -> np.dtype:
        dt = np.dtype(_np_fields(cls), align=True)
        assert dt.itemsize == C.sizeof(cls), (cls.__name__, dt.itemsize, C.sizeof(cls))
        return dt


def _np_fields(cls):
    out = []
    for name, t in cls._fields_:
        out.append((name, _np_type(t)))
    return out


def _np_type(t):
    if hasattr(t, "_fields_"):
        return np.dtype(_np_fields(t), align=True)
    if issubclass(t, C.Array):
        return (_np_type(t._type_), (t._length_,))
    return np.dtype(t)


class DofsFlowParams(C.Structure, _NpMixin):
    """dofs_flow_params: calcOpticalFlowFarneback arguments (cpp/src/segment.cpp:101)."""
    _fields_ = [
        ("pyr_scale", C.c_double),
        ("levels", C.c_int32),
        ("winsize", C.c_int32),
        ("iterations", C.c_int32),
        ("poly_n", C.c_int32),
        ("poly_sigma", C.c_double),
        ("flags", C.c_int32),
    ]


def default_flow_params(**kw) -> "DofsFlowParams":
    p = DofsFlowParams(0.5, 3, 15, 3, 5, 1.2, 0)
    for k, v in kw.items():
        setattr(p, k, v)
    return p


class DofsParams(C.Structure, _NpMixin):
    _fields_ = [
        ("blur_sigma", C.c_double),
        ("neighbor", C.c_int32),
        ("min_size", C.c_int32),
        ("score_threshold", C.c_double),
        ("overlay_min_score", C.c_double),
        ("min_convexity", C.c_double * 3),
        ("obj_size", (C.c_int32 * 2) * 3),
    ]


class DofsSolution(C.Structure, _NpMixin):
    _fields_ = [
        ("cls", C.c_int32),
        ("valid", C.c_int32),
        ("ps_bev", (C.c_float * 2) * 4),
        ("lower_face", (C.c_float * 2) * 4),
        ("upper_face", (C.c_float * 2) * 4),
        ("rectangle", (C.c_float * 2) * 4),
        ("w_error", C.c_double),
        ("h_error", C.c_double),
        ("orient", C.c_double),
    ]


class DofsSnapshot(C.Structure, _NpMixin):
    _fields_ = [
        ("slot", C.c_int32),
        ("event", C.c_int32),
        ("size", C.c_int32),
        ("seg_begin", C.c_int32),
        ("bbox", C.c_int32 * 4),
        ("score", C.c_double),
        ("move", C.c_double),
        ("sol", DofsSolution),
    ]


class DofsStats(C.Structure, _NpMixin):
    _fields_ = [
        ("n_edges", C.c_int64),
        ("n_merges", C.c_int64),
        ("n_candidates", C.c_int64),
        ("n_scored", C.c_int64),
        ("n_qualified", C.c_int64),
        ("n_snapshots", C.c_int64),
    ]


class DofsResult(C.Structure):
    _fields_ = [
        ("snapshots", C.POINTER(DofsSnapshot)),
        ("snapshot_capacity", C.c_int32),
        ("n_snapshots", C.c_int32),
        ("labels", C.POINTER(C.c_int32)),
        ("leaf_order", C.POINTER(C.c_int32)),
        ("blurred", C.POINTER(C.c_float)),
        ("stats", DofsStats),
    ]


class DofsEdge(C.Structure, _NpMixin):
    """Edge (graph.hpp:13-17): {int start; int end; double weight;} — 16 bytes."""
    _fields_ = [
        ("start", C.c_int32),
        ("end", C.c_int32),
        ("weight", C.c_double),
    ]


class DofsEvent(C.Structure, _NpMixin):
    _fields_ = [
        ("start", C.c_int32),
        ("end", C.c_int32),
        ("weight", C.c_double),
        ("root", C.c_int32),
        ("size", C.c_int32),
        ("rank", C.c_int32),
        ("bbox", C.c_int32 * 4),
        ("mean", C.c_float * 2),
    ]


class DofsBoxRecord(C.Structure, _NpMixin):
    _fields_ = [
        ("frame", C.c_int32),
        ("slot", C.c_int32),
        ("cls", C.c_int32),
        ("size", C.c_int32),
        ("score", C.c_double),
        ("move", C.c_double),
        ("lower_face", (C.c_float * 2) * 4),
        ("upper_face", (C.c_float * 2) * 4),
    ]


def default_params() -> DofsParams:
    """Reference constants (graph.hpp:93-94, graph.cpp:328-339, segment.cpp:52,154,166, lifting_3d.cpp:257)."""
    p = DofsParams()
    p.blur_sigma = 3.0
    p.neighbor = 8
    p.min_size = 500
    p.score_threshold = 0.3
    p.overlay_min_score = 0.7
    p.min_convexity[0] = 3.0 / 4.0
    p.min_convexity[1] = 1.0 / 2.0
    p.min_convexity[2] = 20.0 / 29.0
    for c, (l, w) in enumerate(((258, 84), (349, 165), (370, 180))):
        p.obj_size[c][0] = l
        p.obj_size[c][1] = w
    return p


def solution_dict(s) -> dict:
    """DofsSolution (ctypes or numpy record) → plain dict of numpy arrays."""
    get = (lambda k: s[k]) if isinstance(s, np.void) else (lambda k: getattr(s, k))
    out = {"cls": int(get("cls")), "valid": int(get("valid"))}
    for k in ("ps_bev", "lower_face", "upper_face", "rectangle"):
        out[k] = np.array(get(k), dtype=np.float32).reshape(4, 2)
    for k in ("w_error", "h_error", "orient"):
        out[k] = float(get(k))
    return out
