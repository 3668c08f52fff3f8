"""Device context and buffers on top of the C ABI (no torch on the product path).

``Context`` owns one HIP device + stream (``lslam_ctx``).  ``DeviceArray`` is a
typed device allocation with explicit ``upload``/``download``.  One process
per GPU: under ``torch.distributed.run`` pass ``LOCAL_RANK`` as the device.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib


class Context:
    def __init__(self, device: int = 0):
        L = _lib.load()
        self._L = L
        h = C.c_void_p()
        _lib.check(L.lslam_ctx_create(int(device), C.byref(h)), "lslam_ctx_create(%d)" % device)
        self.handle = h
        self.device = int(device)
        self._inflight = []  # host buffers of async copies, held until the next sync()

    @staticmethod
    def device_count() -> int:
        n = C.c_int(0)
        _lib.load().lslam_device_count(C.byref(n))
        return n.value

    def sync(self):
        _lib.check(self._L.lslam_sync(self.handle), "lslam_sync")
        self._inflight.clear()

    def set_timing(self, on: bool = True, kernels=None):
        """HIP-event timing of the kernel ids in ``kernels`` (default: all)."""
        mask = 0xFFFFFFFF if kernels is None else sum(1 << int(k) for k in kernels)
        _lib.check(self._L.lslam_set_timing_mask(self.handle, mask), "lslam_set_timing_mask")
        _lib.check(self._L.lslam_set_timing(self.handle, 1 if on else 0), "lslam_set_timing")

    def timing(self, kernel: int):
        ms = C.c_double(0)
        n = C.c_int64(0)
        _lib.check(self._L.lslam_timing(self.handle, int(kernel), C.byref(ms), C.byref(n)), "lslam_timing")
        return ms.value, n.value

    def timing_reset(self):
        _lib.check(self._L.lslam_timing_reset(self.handle), "lslam_timing_reset")

    def set_steps_budget(self, nbytes: int = 0):
        """Producer steps scratch per slot (bytes; 0 = default 2 GiB).  One-chunk scans whose
        parity-mode steps exceed it run the producer in epochs (lslam_set_steps_budget)."""
        _lib.check(self._L.lslam_set_steps_budget(self.handle, int(nbytes)), "lslam_set_steps_budget")

    @property
    def stream(self):
        """The context's main hipStream_t (int address), for collectives enqueued after its calls."""
        s = C.c_void_p()
        _lib.check(self._L.lslam_ctx_stream(self.handle, C.byref(s)), "lslam_ctx_stream")
        return s.value or 0

    def copy(self, dst, src, nbytes=None):
        """Device-to-device copy on the context stream (async)."""
        n = dst.nbytes if nbytes is None else int(nbytes)
        _lib.check(self._L.lslam_d2d(self.handle, dst.ptr if isinstance(dst, DeviceArray) else C.c_void_p(dst),
                                     src.ptr if isinstance(src, DeviceArray) else C.c_void_p(src), n), "lslam_d2d")

    def empty(self, shape, dtype):
        return DeviceArray(self, shape, dtype)

    def to_device(self, arr):
        arr = np.ascontiguousarray(arr)
        d = DeviceArray(self, arr.shape, arr.dtype)
        d.upload(arr)
        return d

    def close(self):
        if self.handle:
            self._L.lslam_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class DeviceArray:
    def __init__(self, ctx: Context, shape, dtype):
        self.ctx = ctx
        self.shape = tuple(int(s) for s in (shape if isinstance(shape, (tuple, list)) else (shape,)))
        self.dtype = np.dtype(dtype)
        self.nbytes = int(np.prod(self.shape, dtype=np.int64)) * self.dtype.itemsize
        p = C.c_void_p()
        _lib.check(ctx._L.lslam_malloc(ctx.handle, max(self.nbytes, 16), C.byref(p)), "lslam_malloc")
        self.ptr = p

    @property
    def addr(self):
        return self.ptr.value

    def upload(self, arr):
        arr = np.ascontiguousarray(arr, dtype=self.dtype)
        if arr.nbytes != self.nbytes:
            raise ValueError("upload size mismatch %d != %d" % (arr.nbytes, self.nbytes))
        _lib.check(self.ctx._L.lslam_h2d(self.ctx.handle, self.ptr, arr.ctypes.data_as(C.c_void_p),
                                         self.nbytes), "lslam_h2d")
        self.ctx._inflight.append(arr)  # a caller's temporary must outlive the copy
        self.ctx.sync()  # arr may be a temporary: finish before it is freed

    def upload_async(self, arr):
        """H2D on the context stream without waiting: ``arr`` (ideally page-locked, see
        ``register_host``) must stay alive and unchanged until the next ``ctx.sync()``."""
        if not (isinstance(arr, np.ndarray) and arr.flags.c_contiguous and arr.dtype == self.dtype):
            raise ValueError("upload_async needs a C-contiguous %s array" % self.dtype)
        if arr.nbytes != self.nbytes:
            raise ValueError("upload size mismatch %d != %d" % (arr.nbytes, self.nbytes))
        _lib.check(self.ctx._L.lslam_h2d(self.ctx.handle, self.ptr, arr.ctypes.data_as(C.c_void_p),
                                         self.nbytes), "lslam_h2d")
        self.ctx._inflight.append(arr)  # held until the next sync(), whoever else drops it

    def download_async(self, out):
        """D2H on the context stream without waiting: ``out`` (a C-contiguous host array of
        the same size, ideally page-locked) holds the data after the next ``ctx.sync()``."""
        if not (isinstance(out, np.ndarray) and out.flags.c_contiguous and out.nbytes == self.nbytes):
            raise ValueError("download_async needs a C-contiguous host array of %d bytes" % self.nbytes)
        _lib.check(self.ctx._L.lslam_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p), self.ptr, self.nbytes),
                   "lslam_d2h")
        self.ctx._inflight.append(out)

    def download(self, out=None):
        if out is None:
            out = np.empty(self.shape, self.dtype)
        _lib.check(self.ctx._L.lslam_d2h(self.ctx.handle, out.ctypes.data_as(C.c_void_p), self.ptr,
                                         self.nbytes), "lslam_d2h")
        self.ctx.sync()
        return out

    def fill_zero(self):
        _lib.check(self.ctx._L.lslam_memset(self.ctx.handle, self.ptr, 0, self.nbytes), "lslam_memset")

    def free(self):
        if self.ptr and self.ptr.value:
            self.ctx._L.lslam_free(self.ctx.handle, self.ptr)
            self.ptr = C.c_void_p()

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass


def ptr(x):
    """Device address of a DeviceArray (or None)."""
    return None if x is None else x.addr


def register_host(arr) -> bool:
    """Page-lock a host array in place (hipHostRegister); False if the runtime refuses."""
    return _lib.load().lslam_host_register(arr.ctypes.data_as(C.c_void_p), arr.nbytes) == _lib.LSLAM_OK


def unregister_host(arr):
    _lib.load().lslam_host_unregister(arr.ctypes.data_as(C.c_void_p))
