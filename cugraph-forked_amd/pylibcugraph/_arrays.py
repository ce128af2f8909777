"""Device-array plumbing between Python objects and libcugraph_c views.

The reference accepts ``__cuda_array_interface__`` objects (cupy/cudf) and returns
cupy arrays (``utils.pyx:150-184``).  cupy/cudf do not exist on ROCm here, so
this build accepts torch tensors (any device), numpy arrays / lists / pandas
Series (copied to HBM) and ``__cuda_array_interface__`` objects, and returns
torch tensors resident on the GPU.  torch is plumbing only: every computation
happens in libcugraph_c.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _lib

_NP_TO_C = {np.dtype(np.int32): _lib.INT32, np.dtype(np.int64): _lib.INT64,
            np.dtype(np.float32): _lib.FLOAT32, np.dtype(np.float64): _lib.FLOAT64}
_C_TO_NP = {v: k for k, v in _NP_TO_C.items()}


def _torch():
    import torch
    return torch


def _torch_dtype(c_type):
    torch = _torch()
    return {_lib.INT32: torch.int32, _lib.INT64: torch.int64,
            _lib.FLOAT32: torch.float32, _lib.FLOAT64: torch.float64}[c_type]


def _c_type_of_torch(t):
    torch = _torch()
    m = {torch.int32: _lib.INT32, torch.int64: _lib.INT64,
         torch.float32: _lib.FLOAT32, torch.float64: _lib.FLOAT64}
    if t.dtype not in m:
        raise TypeError(f"unsupported dtype {t.dtype}")
    return m[t.dtype]


def to_device_tensor(arr, dtype=None):
    """Return a contiguous GPU torch tensor for ``arr`` (no copy if already one)."""
    torch = _torch()
    if isinstance(arr, torch.Tensor):
        t = arr
    elif hasattr(arr, "__cuda_array_interface__") and not isinstance(arr, np.ndarray):
        t = torch.as_tensor(arr, device="cuda")
    else:
        if hasattr(arr, "to_numpy"):
            arr = arr.to_numpy()
        t = torch.from_numpy(np.ascontiguousarray(np.asarray(arr)))
    if dtype is not None:
        t = t.to(dtype)
    if not t.is_cuda:
        t = t.to("cuda")
    return t.contiguous()


class DeviceView:
    """Owns a ``cugraph_type_erased_device_array_view_t*`` plus the tensor it wraps."""

    def __init__(self, arr, dtype=None):
        self.tensor = to_device_tensor(arr, dtype)
        self.c_type = _c_type_of_torch(self.tensor)
        self.ptr = _lib.lib.cugraph_type_erased_device_array_view_create(
            ctypes.c_void_p(self.tensor.data_ptr()), self.tensor.numel(), self.c_type)

    def __del__(self, _sd=_lib.SHUTDOWN, _free=_lib.lib.cugraph_type_erased_device_array_view_free):
        if getattr(self, "ptr", None) and not _sd[0]:
            _free(self.ptr)
            self.ptr = None


def optional_view(arr, dtype=None):
    return None if arr is None else DeviceView(arr, dtype)


def vptr(v):
    return None if v is None else v.ptr


def copy_view_to_tensor(handle_ptr, view_ptr, free_view=True):
    """utils.pyx:150-184 copy_to_cupy_array, returning a torch tensor on the GPU."""
    torch = _torch()
    c_type = _lib.lib.cugraph_type_erased_device_array_view_type(view_ptr)
    n = _lib.lib.cugraph_type_erased_device_array_view_size(view_ptr)
    out = torch.empty(n, dtype=_torch_dtype(c_type), device="cuda")
    dst = _lib.lib.cugraph_type_erased_device_array_view_create(ctypes.c_void_p(out.data_ptr()), n, c_type)
    try:
        _lib.call("cugraph_type_erased_device_array_view_copy", handle_ptr, dst, view_ptr)
    finally:
        _lib.lib.cugraph_type_erased_device_array_view_free(dst)
        if free_view:
            _lib.lib.cugraph_type_erased_device_array_view_free(view_ptr)
    return out


def copy_views_to_tensors(handle_ptr, view_ptrs):
    """copy_view_to_tensor for several result views with one C call (one stream
    synchronize instead of one per array); the source views are freed."""
    torch = _torch()
    outs, dsts = [], []
    try:
        for v in view_ptrs:
            c_type = _lib.lib.cugraph_type_erased_device_array_view_type(v)
            n = _lib.lib.cugraph_type_erased_device_array_view_size(v)
            out = torch.empty(n, dtype=_torch_dtype(c_type), device="cuda")
            outs.append(out)
            dsts.append(_lib.lib.cugraph_type_erased_device_array_view_create(ctypes.c_void_p(out.data_ptr()), n,
                                                                               c_type))
        k = len(view_ptrs)
        dst_arr = (ctypes.c_void_p * k)(*dsts)
        src_arr = (ctypes.c_void_p * k)(*view_ptrs)
        _lib.call("cugraph_amd_device_array_views_copy", handle_ptr, k, ctypes.cast(dst_arr, ctypes.c_void_p),
                  ctypes.cast(src_arr, ctypes.c_void_p))
    finally:
        for d in dsts:
            _lib.lib.cugraph_type_erased_device_array_view_free(d)
        for v in view_ptrs:
            _lib.lib.cugraph_type_erased_device_array_view_free(v)
    return outs


_TYPESTR = {_lib.INT32: "<i4", _lib.INT64: "<i8", _lib.FLOAT32: "<f4", _lib.FLOAT64: "<f8"}


class ResultOwner:
    """Keeps a libcugraph_c result -- and the device arrays it owns -- alive while
    tensors view its arrays; frees it when the last of them is gone.  The free
    returns the memory to the library's stream-ordered cache, which reuses blocks
    without waiting on other streams, so the whole device that owns the arrays is
    synchronised first: no reader on any stream (torch's current one, a side
    stream, another device's current stream) can still be running when the
    library reuses the block."""

    def __init__(self, ptr, free_fn):
        self.ptr = ptr
        self._free = free_fn
        self._device = _torch().cuda.current_device()

    def __del__(self, _sd=_lib.SHUTDOWN):
        if getattr(self, "ptr", None) and not _sd[0]:
            try:
                _torch().cuda.synchronize(self._device)
            finally:
                self._free(self.ptr)
                self.ptr = None


class _OwnedDeviceArray:
    """``__cuda_array_interface__`` over one result array; holds the owner."""

    def __init__(self, owner, ptr, n, c_type):
        self._owner = owner
        self.__cuda_array_interface__ = {"shape": (n,), "typestr": _TYPESTR[c_type], "data": (ptr, False),
                                         "strides": None, "version": 3}


def views_to_tensors_owned(handle_ptr, view_ptrs, res_ptr, free_fn):
    """Result views -> GPU torch tensors WITHOUT a copy (the reference's
    copy_to_cupy_array copies; here the tensors view the library's result arrays and
    keep the result alive through a ResultOwner).  One stream synchronize; the
    views are freed, the result is freed when the tensors are."""
    torch = _torch()
    owner = ResultOwner(res_ptr, free_fn)
    outs = []
    try:
        _lib.call("cugraph_amd_device_array_views_copy", handle_ptr, 0, None, None)  # handle stream synchronize
        for v in view_ptrs:
            c_type = _lib.lib.cugraph_type_erased_device_array_view_type(v)
            n = _lib.lib.cugraph_type_erased_device_array_view_size(v)
            ptr = _lib.lib.cugraph_type_erased_device_array_view_pointer(v)
            if n == 0 or not ptr:
                outs.append(torch.empty(0, dtype=_torch_dtype(c_type), device="cuda"))
            else:
                outs.append(torch.as_tensor(_OwnedDeviceArray(owner, ptr, n, c_type), device="cuda"))
    finally:
        for v in view_ptrs:
            _lib.lib.cugraph_type_erased_device_array_view_free(v)
    return outs


def copy_view_to_numpy(handle_ptr, view_ptr):
    c_type = _lib.lib.cugraph_type_erased_device_array_view_type(view_ptr)
    n = _lib.lib.cugraph_type_erased_device_array_view_size(view_ptr)
    out = np.empty(n, dtype=_C_TO_NP[c_type])
    _lib.call("cugraph_type_erased_device_array_view_copy_to_host", handle_ptr,
              out.ctypes.data_as(ctypes.c_void_p), view_ptr)
    return out


class DeviceArray:
    """Owning ``cugraph_type_erased_device_array_t*`` returned by the extensions."""

    def __init__(self, ptr):
        self.ptr = ptr

    def view(self):
        return _lib.lib.cugraph_type_erased_device_array_view(self.ptr)

    def to_tensor(self, handle_ptr):
        return copy_view_to_tensor(handle_ptr, self.view())

    def __len__(self):
        v = self.view()
        n = _lib.lib.cugraph_type_erased_device_array_view_size(v)
        _lib.lib.cugraph_type_erased_device_array_view_free(v)
        return n

    def __del__(self, _sd=_lib.SHUTDOWN, _free=_lib.lib.cugraph_type_erased_device_array_free):
        if getattr(self, "ptr", None) and not _sd[0]:
            _free(self.ptr)
            self.ptr = None
