"""Buffer normalisation for host buffers and HIP device tensors.

Reference semantics: src/numcodecs/compat.py:9-206 (``ensure_ndarray_like``,
``ensure_contiguous_ndarray``, ``ensure_bytes``, ``ndarray_copy``).  The
reference only understands the buffer protocol (and, nominally, CuPy through
its ``NDArrayLike`` protocol); PyTorch tensors satisfy neither.  This module
adds device tensors as first-class citizens:

* a ``torch.Tensor`` on a HIP device stays on the device -- codecs return
  device tensors;
* everything else is normalised exactly as the reference does (numpy views,
  object arrays rejected, datetime viewed as int64, non-contiguous rejected),
  then staged to the device through pinned memory, processed there, and
  brought back as numpy -- the arithmetic never runs on the host.

``DBuf`` is the internal currency: a flat contiguous ``torch.uint8`` device
tensor of raw bytes plus the numpy dtype, shape and memory order it stands
for.
"""

from __future__ import annotations

import array
from dataclasses import dataclass

import numpy as np
import torch

from . import _native, _ops

__all__ = [
    "DBuf",
    "ensure_ndarray_like",
    "is_ndarray_like",
    "ensure_ndarray",
    "ensure_contiguous_ndarray",
    "ensure_bytes",
    "ndarray_copy",
    "is_device_tensor",
    "torch_dtype",
    "numpy_dtype",
]

# numpy dtype.str <-> torch dtype (little-endian / byte-sized types)
_NP_TO_TORCH = {
    "|b1": torch.bool,
    "|i1": torch.int8,
    "<i2": torch.int16,
    "<i4": torch.int32,
    "<i8": torch.int64,
    "|u1": torch.uint8,
    "<u2": torch.uint16,
    "<u4": torch.uint32,
    "<u8": torch.uint64,
    "<f2": torch.float16,
    "<f4": torch.float32,
    "<f8": torch.float64,
    "<c8": torch.complex64,
    "<c16": torch.complex128,
}
_TORCH_TO_NP = {v: np.dtype(k) for k, v in _NP_TO_TORCH.items()}


def torch_dtype(dt) -> "torch.dtype | None":
    """torch dtype with the same bytes as numpy dtype `dt` (None if none)."""
    return _NP_TO_TORCH.get(np.dtype(dt).str)


def numpy_dtype(tdt: torch.dtype) -> np.dtype:
    try:
        return _TORCH_TO_NP[tdt]
    except KeyError:
        raise TypeError(f"tensor dtype {tdt} has no numpy equivalent supported here") from None


def is_device_tensor(x) -> bool:
    return isinstance(x, torch.Tensor) and x.device.type == "cuda"


# ---------------------------------------------------------------------------
# host-side normalisation: the reference semantics, verbatim in behaviour
# ---------------------------------------------------------------------------
# DLPack device types of a HIP device array (dlpack.h: kDLCUDA = 2, kDLROCM = 10)
_DL_DEVICE_TYPES = (2, 10)


def _device_array_as_tensor(buf) -> "torch.Tensor | None":
    """A zero-copy torch view of a NON-torch array living in HIP device memory
    (CuPy-style ``__cuda_array_interface__`` or a DLPack producer whose
    ``__dlpack_device__`` is a GPU), else None.  This is the device half of
    the reference's NDArrayLike hook (ndarray_like.py:39-60,
    compat.py:32-33: an ndarray-like object is used as it is)."""
    dev = getattr(buf, "__dlpack_device__", None)
    if dev is not None and hasattr(buf, "__dlpack__"):
        try:
            dtype_code = int(dev()[0])
        except Exception:
            return None
        if dtype_code in _DL_DEVICE_TYPES:
            return torch.from_dlpack(buf)
        return None
    if hasattr(buf, "__cuda_array_interface__"):
        # no device argument: torch takes the device the pointer lives on, so
        # an array on another GPU is viewed there, never copied
        return torch.as_tensor(buf)
    return None


_OWN_TYPES = (torch.Tensor, np.ndarray, bytes, bytearray, memoryview, array.array)


def device_out(out):
    """`out` as this module handles it: another library's device array
    (DLPack / ``__cuda_array_interface__``) becomes a zero-copy torch view of
    its memory, so results are written into the caller's buffer in place;
    anything else is returned unchanged."""
    if out is None or isinstance(out, _OWN_TYPES):
        return out
    dt = _device_array_as_tensor(out)
    return out if dt is None else dt


def is_ndarray_like(obj) -> bool:
    """ndarray_like.py:39-64: True for objects with the ndarray attributes the
    reference's NDArrayLike protocol lists (numpy arrays, CuPy-like device
    arrays); torch tensors on a HIP device are accepted everywhere too."""
    if isinstance(obj, (np.ndarray, torch.Tensor)):
        return True
    needed = ("dtype", "shape", "strides", "ndim", "size", "itemsize", "nbytes", "flags", "__len__",
              "__getitem__", "__setitem__", "tobytes", "reshape", "view")
    return all(hasattr(obj, a) for a in needed)


def ensure_ndarray_like(buf):
    """compat.py:9-41 -- a view of `buf` (numpy array or device tensor).
    Device arrays of other libraries (DLPack / ``__cuda_array_interface__``)
    become zero-copy device tensors."""
    if is_device_tensor(buf):
        return buf
    if isinstance(buf, torch.Tensor):  # CPU tensor: the numpy view of it
        return buf.detach().numpy()
    if isinstance(buf, np.ndarray):
        return buf
    dt = _device_array_as_tensor(buf)
    if dt is not None:
        return dt
    if isinstance(buf, array.array) and buf.typecode in "cu":
        raise TypeError("array.array with char or unicode type is not supported")
    return np.array(memoryview(buf), copy=False)


def ensure_ndarray(buf):
    """compat.py:44-63."""
    a = ensure_ndarray_like(buf)
    return a if is_device_tensor(a) else np.asarray(a)


def _tensor_order(t: torch.Tensor) -> "str | None":
    """'C' / 'F' if `t` covers contiguous memory in that order, else None."""
    if t.is_contiguous():
        return "C"
    if t.dim() >= 2 and t.permute(*reversed(range(t.dim()))).is_contiguous():
        return "F"
    return None


def ensure_contiguous_ndarray(buf, max_buffer_size=None, flatten=True):
    """compat.py:66-150 -- flat (memory-order) contiguous view, host or device."""
    arr = ensure_ndarray_like(buf)
    if is_device_tensor(arr):
        order = _tensor_order(arr)
        if order is None:
            raise ValueError("an array with contiguous memory is required")
        if flatten:
            arr = arr.reshape(-1) if order == "C" else arr.permute(*reversed(range(arr.dim()))).reshape(-1)
        nbytes = arr.numel() * arr.element_size()
    else:
        arr = np.asarray(arr)
        if arr.dtype == object:
            raise TypeError("object arrays are not supported")
        if arr.dtype.kind in "Mm":
            arr = arr.view(np.int64)
        if arr.flags.c_contiguous or arr.flags.f_contiguous:
            if flatten:
                arr = arr.reshape(-1, order="A")
        else:
            raise ValueError("an array with contiguous memory is required")
        nbytes = arr.nbytes
    if max_buffer_size is not None and nbytes > max_buffer_size:
        raise ValueError(f"Codec does not support buffers of > {max_buffer_size} bytes")
    return arr


def ensure_bytes(buf) -> bytes:
    """compat.py:153-167 (device tensors are downloaded)."""
    if isinstance(buf, bytes):
        return buf
    if is_device_tensor(buf):
        return ensure_contiguous_ndarray(buf).view(torch.uint8).cpu().numpy().tobytes()
    arr = ensure_ndarray_like(buf)
    if arr.dtype == object:
        raise TypeError("object arrays are not supported")
    return arr.tobytes(order="A")


# ---------------------------------------------------------------------------
# device staging
# ---------------------------------------------------------------------------
def _device() -> torch.device:
    _native.require_device()
    return torch.device("cuda", torch.cuda.current_device())


def upload(host: np.ndarray, device=None) -> torch.Tensor:
    """Contiguous host array -> flat uint8 device tensor (pinned staging)."""
    device = device if device is not None else _device()
    src = host.reshape(-1, order="A").view(np.uint8) if host.ndim else host.reshape(1).view(np.uint8)
    n = src.nbytes
    if n == 0:
        return torch.empty(0, dtype=torch.uint8, device=device)
    stage = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    np.copyto(stage.numpy(), src)
    return stage.to(device, non_blocking=True)


def download(dev: torch.Tensor) -> np.ndarray:
    """Flat uint8 device tensor -> host uint8 numpy array (owns its memory)."""
    n = dev.numel()
    if n == 0:
        return np.empty(0, dtype=np.uint8)
    host = torch.empty(n, dtype=torch.uint8, pin_memory=True)
    host.copy_(dev, non_blocking=True)
    torch.cuda.current_stream(dev.device).synchronize()
    return host.numpy()


_U8 = np.dtype(np.uint8)


@dataclass
class DBuf:
    """Raw bytes on the device + the numpy array they stand for."""

    data: torch.Tensor  # flat, contiguous, torch.uint8, on a HIP device
    dtype: np.dtype
    shape: tuple
    order: str  # 'C' or 'F': memory order of `shape`
    host: bool  # True when the caller handed us a host buffer

    @property
    def nbytes(self) -> int:
        return self.data.numel()

    @property
    def count(self) -> int:
        return self.nbytes // max(self.dtype.itemsize, 1)

    def ptr(self) -> int:
        return self.data.data_ptr()

    def with_dtype(self, dtype, shape=None, order=None) -> "DBuf":
        dtype = np.dtype(dtype)
        if shape is None:
            shape = (self.nbytes // dtype.itemsize,)
        return DBuf(self.data, dtype, tuple(shape), order or "C", self.host)


def to_dbuf(buf, *, flatten=True, contiguous=True) -> DBuf:
    """Normalise any accepted input to a DBuf.

    Host inputs follow ``ensure_contiguous_ndarray`` (contiguous=True) or
    ``ensure_ndarray`` (contiguous=False: a non-contiguous array is copied in
    C order, as the reference's ``reshape(-1, order='A')`` would) and are
    uploaded; device tensors are used in place.
    """
    if (type(buf) is torch.Tensor and buf.dtype is torch.uint8 and buf.dim() == 1 and buf.is_cuda
            and buf.is_contiguous()):
        # the common case (an encoded chunk): flat device bytes, used as they are
        return DBuf(buf, _U8, (buf.numel(),), "C", False)
    if type(buf) is torch.Tensor and buf.is_cuda and buf.is_contiguous() and buf.numel():
        # a C-contiguous device array (a chunk to encode): its bytes in place
        dtype = _TORCH_TO_NP.get(buf.dtype)
        if dtype is not None:
            shape = (buf.numel(),) if flatten else tuple(buf.shape)
            return DBuf(buf.view(-1).view(torch.uint8), dtype, shape, "C", False)
    if not isinstance(buf, (torch.Tensor, np.ndarray, bytes, bytearray, memoryview)):
        dt = _device_array_as_tensor(buf)  # another library's device array: in place
        if dt is not None:
            buf = dt
    if is_device_tensor(buf):
        order = _tensor_order(buf)
        if order is None:
            if contiguous:
                raise ValueError("an array with contiguous memory is required")
            buf = buf.contiguous()
            order = "C"
        dtype = numpy_dtype(buf.dtype)
        shape = tuple(buf.shape)
        flat = buf.reshape(-1) if order == "C" else buf.permute(*reversed(range(buf.dim()))).reshape(-1)
        raw = flat.view(torch.uint8) if flat.numel() else flat.new_empty(0, dtype=torch.uint8)
        if flatten:
            shape = (flat.numel(),)
            order = "C"
        return DBuf(raw, dtype, shape, order, False)
    if contiguous:
        arr = ensure_contiguous_ndarray(buf, flatten=False)
    else:
        arr = np.asarray(ensure_ndarray(buf))
        if arr.dtype == object:
            raise TypeError("object arrays are not supported")
        if not (arr.flags.c_contiguous or arr.flags.f_contiguous):
            arr = np.ascontiguousarray(arr)
    order = "F" if (arr.flags.f_contiguous and not arr.flags.c_contiguous) else "C"
    shape = (arr.size,) if flatten else arr.shape
    if flatten:
        order = "C"
    return DBuf(upload(arr), arr.dtype, tuple(shape), order, True)


def empty_like_bytes(nbytes: int, like: DBuf) -> torch.Tensor:
    return torch.empty(nbytes, dtype=torch.uint8, device=like.data.device)


def device_out_bytes(out, nbytes: int, like: "DBuf | torch.Tensor") -> "torch.Tensor | None":
    """The raw bytes of a caller's device `out` when a decode kernel can write
    its result there directly instead of into a temporary that
    :func:`ndarray_copy` then copies (same device as the input, contiguous in
    C or F order, exactly `nbytes`, 16-B aligned, not overlapping the input):
    the bytes land exactly where ndarray_copy would put them.  None sends
    the result through ndarray_copy, which raises the reference's errors for
    the other cases."""
    data = like.data if isinstance(like, DBuf) else like  # the input's bytes
    out = device_out(out)
    if out is None or not is_device_tensor(out) or out.device != data.device or nbytes == 0:
        return None
    order = _tensor_order(out)
    if order is None:
        return None
    flat = out.reshape(-1) if order == "C" else out.permute(*reversed(range(out.dim()))).reshape(-1)
    if flat.numel() * flat.element_size() != nbytes:
        return None
    raw = flat.view(torch.uint8)
    p, q = raw.data_ptr(), data.data_ptr()
    if p % 16 or (p < q + data.numel() * data.element_size() and q < p + nbytes):
        return None
    return raw


def finish(raw: torch.Tensor, dtype, shape, order: str, host: bool):
    """Present device bytes as the caller's kind of array.

    host=True: a numpy array of `dtype`/`shape`/`order`; otherwise a device
    tensor view with the torch dtype (uint8 bytes when torch lacks the dtype).
    """
    dtype = np.dtype(dtype)
    shape = tuple(shape)
    if host:
        a = download(raw).view(dtype)
        return a.reshape(shape, order=order)
    tdt = torch_dtype(dtype)
    if tdt is None:  # no torch equivalent (e.g. big-endian): raw bytes
        return raw
    t = raw.view(tdt) if raw.numel() else torch.empty(0, dtype=tdt, device=raw.device)
    if order == "F" and len(shape) >= 2:
        return t.reshape(tuple(reversed(shape))).permute(*reversed(range(len(shape))))
    return t.reshape(shape)


def ndarray_copy(src, dst):
    """compat.py:177-206 -- copy `src` into `dst` (host or device, either way).

    `src` is the codec's result (numpy array or device tensor).  Returns `dst`
    as numcodecs does (the normalised view of it).
    """
    if dst is None:
        return src
    dt = device_out(dst)  # another library's device array: write into its memory
    if dt is not dst:
        ndarray_copy(src, dt)
        return dst
    if is_device_tensor(dst):
        order = _tensor_order(dst)
        if order is None:
            raise ValueError("an array with contiguous memory is required")
        d_flat = dst.reshape(-1) if order == "C" else dst.permute(*reversed(range(dst.dim()))).reshape(-1)
        d_raw = d_flat.view(torch.uint8) if d_flat.numel() else d_flat.new_empty(0, dtype=torch.uint8)
        if is_device_tensor(src):
            s_raw = ensure_contiguous_ndarray(src)
            s_raw = s_raw.view(torch.uint8) if s_raw.numel() else s_raw.new_empty(0, dtype=torch.uint8)
        else:
            s_raw = upload(np.ascontiguousarray(src))
        if s_raw.numel() != d_raw.numel():
            raise ValueError(
                f"cannot copy {s_raw.numel()} bytes into an output buffer of {d_raw.numel()} bytes"
            )
        if s_raw.device == d_raw.device:
            _ops.copy(s_raw, d_raw, s_raw.numel())
        else:
            d_raw.copy_(s_raw)
        return dst
    # host destination
    d = ensure_ndarray_like(dst)
    if is_device_tensor(src):
        s = ensure_contiguous_ndarray(src)
        s = download(s.view(torch.uint8) if s.numel() else s.new_empty(0, dtype=torch.uint8))
    else:
        s = ensure_ndarray_like(src).reshape(-1, order="A")
    if d.dtype != object:
        s = s.view(d.dtype)
    if s.shape != d.shape:
        s = s.reshape(d.shape, order="F" if d.flags.f_contiguous else "C")
    np.copyto(d, s)
    return d
