"""MI355X build extensions: device R-MAT generator and cugraph.Graph edge-list
preprocessing (include/cugraph_amd/ext.h).

``generate_rmat_edgelist`` plays the role of the reference's
``cugraph.generators.rmat`` (RAFT generator,
``cpp/src/generators/generate_rmat_edgelist.cu:36-103``) with our own
counter-based stream (definition and numpy twin: ``oracle/rmat.py``).
"""
from __future__ import annotations

import ctypes

from . import _lib
from ._arrays import DeviceArray, DeviceView, optional_view, vptr


def generate_rmat_edgelist(resource_handle, scale, num_edges, a=0.57, b=0.19, c=0.19, seed=42,
                           clip_and_flip=False, scramble_vertex_ids=True, first_edge=0,
                           vertex_dtype="int32"):
    """Returns (src, dst) GPU tensors."""
    vt = _lib.INT32 if str(vertex_dtype).endswith("int32") else _lib.INT64
    s, d = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.call("cugraph_amd_generate_rmat_edgelist", resource_handle.ptr, int(scale), int(num_edges),
              float(a), float(b), float(c), int(seed), int(bool(clip_and_flip)),
              int(bool(scramble_vertex_ids)), int(first_edge), vt, ctypes.byref(s), ctypes.byref(d))
    h = resource_handle.ptr
    return DeviceArray(s.value).to_tensor(h), DeviceArray(d.value).to_tensor(h)


def generate_edge_weights(resource_handle, num_edges, seed=42, first_edge=0, weight_dtype="float32"):
    wt = _lib.FLOAT32 if str(weight_dtype).endswith("float32") else _lib.FLOAT64
    w = ctypes.c_void_p()
    _lib.call("cugraph_amd_generate_edge_weights", resource_handle.ptr, int(num_edges), int(seed),
              int(first_edge), wt, ctypes.byref(w))
    return DeviceArray(w.value).to_tensor(resource_handle.ptr)


def symmetrize_dedup(resource_handle, src, dst, weights=None, symmetrize=True):
    """symmetrize.py:78-93 on the device: (src, dst, weights|None) sorted by (src, dst)."""
    sv = DeviceView(src)
    dv = DeviceView(dst, sv.tensor.dtype)
    wv = optional_view(weights)
    so, do, wo = ctypes.c_void_p(), ctypes.c_void_p(), ctypes.c_void_p()
    _lib.call("cugraph_amd_symmetrize_dedup", resource_handle.ptr, sv.ptr, dv.ptr, vptr(wv),
              int(bool(symmetrize)), ctypes.byref(so), ctypes.byref(do), ctypes.byref(wo))
    h = resource_handle.ptr
    return (DeviceArray(so.value).to_tensor(h), DeviceArray(do.value).to_tensor(h),
            DeviceArray(wo.value).to_tensor(h) if wo.value else None)
