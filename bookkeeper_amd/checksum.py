"""Host-side mirror of circe-checksum's checksum facade, backed by the GPU engine.

Reference surface (circe-checksum/src/main/java/com/scurrilous/circe/):
  * ``IntHash`` (checksum/IntHash.java:23-35): calculate / resume / acceptsMemoryAddressBuffer.
  * ``JniIntHash`` (checksum/JniIntHash.java:25-64): the provider ``Crc32cIntChecksum`` selects
    when the native library loads; ``GpuIntHash`` below is its drop-in, reaching
    libbkdigest.so instead of libcirce-checksum.so.
  * ``Crc32cIntChecksum`` (checksum/Crc32cIntChecksum.java:24-100): the static facade that
    bookkeeper-server calls (CRC32CDigestManager.java:49-56).
  * Bounds/argument errors follow AbstractIncrementalIntHash.java:62-69
    (negative length -> IllegalArgumentException ~ ValueError; range -> IndexOutOfBounds ~ IndexError).

Values returned by the per-call API are Java ``int`` bit patterns (signed 32-bit), exactly what
the reference returns; the batch API returns uint32 arrays.

Buffers: ``bytes``/``bytearray``/``memoryview``/numpy arrays are host buffers (the reference's
``byte[]`` / direct ``ByteBuf``); ``torch`` tensors on a HIP device are device-resident buffers
(the new batch path). There is no CPU arithmetic in this module: host buffers go to
``bkd_resume_host`` (the library's native CPU route for small buffers or without a device, the
GPU above ``cpu_route_max``), device tensors to ``bkd_resume_device`` on the tensor's current
stream, so a resume is ordered after the kernels that wrote the tensor.
"""
from __future__ import annotations

import contextlib
import ctypes

import numpy as np

from . import _native
from ._native import CRC32, CRC32C, check, lib

__all__ = ["CRC32C", "CRC32", "GpuIntHash", "Crc32cIntChecksum", "crc_batch", "crc_batch_uniform",
           "crc_batch_segments", "crc_batch_host", "release_stream", "cpu_resume", "set_cpu_route_max", "to_java_int"]


def to_java_int(v: int) -> int:
    v &= 0xFFFFFFFF
    return v - (1 << 32) if v & 0x80000000 else v


def _is_torch_tensor(x) -> bool:
    return type(x).__module__.startswith("torch") and hasattr(x, "data_ptr")


def _stream_ptr(stream, tensor=None):
    """The HIP stream a call is enqueued on: `stream` if given (a torch.cuda.Stream on the tensor's
    device, or a raw handle), else the tensor device's current stream. The library runs the call on
    that stream's device; for the null stream, on the current device, which _on_device sets."""
    if stream is not None:
        sdev = getattr(stream, "device", None)
        if sdev is not None and tensor is not None and _is_torch_tensor(tensor) and tensor.is_cuda \
                and sdev != tensor.device:
            raise ValueError(f"stream is on {sdev} but the buffer is on {tensor.device}")
        return ctypes.c_void_p(int(getattr(stream, "cuda_stream", stream)))
    if tensor is not None and _is_torch_tensor(tensor) and tensor.is_cuda:
        import torch
        return ctypes.c_void_p(int(torch.cuda.current_stream(tensor.device).cuda_stream))
    return ctypes.c_void_p(0)


def _on_device(tensor):
    """Makes the tensor's device current for the call (the null stream runs on the current device)."""
    if _is_torch_tensor(tensor) and tensor.is_cuda:
        import torch
        return torch.cuda.device(tensor.device)
    return contextlib.nullcontext()


def _host_view(buf) -> np.ndarray:
    if isinstance(buf, np.ndarray):
        return np.ascontiguousarray(buf).view(np.uint8).reshape(-1)
    return np.frombuffer(memoryview(buf).cast("B"), dtype=np.uint8)


class GpuIntHash:
    """``IntHash`` implementation whose arithmetic runs in libbkdigest.so (JniIntHash.java:25-64)."""

    def __init__(self, algo: int = CRC32C):
        if algo not in (CRC32C, CRC32):
            raise ValueError("unknown algorithm")
        self.algo = algo
        lib()  # fail loudly now if the HIP library is absent

    # IntHash.calculate(ByteBuf) / calculate(ByteBuf, offset, len)  (IntHash.java:24-26)
    def calculate(self, buffer, offset: int | None = None, length: int | None = None) -> int:
        return self.resume(0, buffer, offset, length)

    # IntHash.resume(int, ByteBuf[, offset, len]) / resume(int, byte[], offset, len)  (IntHash.java:28-32)
    def resume(self, current: int, buffer, offset: int | None = None, length: int | None = None) -> int:
        if offset is None:
            offset = 0
            length = (buffer.numel() * buffer.element_size()) if _is_torch_tensor(buffer) else len(_host_view(buffer))
        elif length is None:
            raise TypeError("offset given without length")
        if length < 0:
            raise ValueError("negative length")  # IllegalArgumentException, AbstractIncrementalIntHash.java:64-65
        out = ctypes.c_uint32(0)
        if _is_torch_tensor(buffer):
            total = buffer.numel() * buffer.element_size()
            if offset < 0 or offset + length > total:
                raise IndexError("range outside buffer")  # AbstractIncrementalIntHash.java:66-67
            if not buffer.is_contiguous():
                raise ValueError("device buffer must be contiguous")
            if not buffer.is_cuda:  # a CPU tensor is a host buffer
                return self.resume(current, buffer.numpy(), offset, length)
            ptr = ctypes.c_void_p(buffer.data_ptr() + offset)
            with _on_device(buffer):
                check(lib().bkd_resume_device(self.algo, current & 0xFFFFFFFF, ptr, length,
                                              _stream_ptr(None, buffer), ctypes.byref(out)))
        else:
            view = _host_view(buffer)
            if offset < 0 or offset + length > view.size:
                raise IndexError("range outside buffer")
            ptr = ctypes.c_void_p(view.ctypes.data + offset) if view.size else ctypes.c_void_p(0)
            check(lib().bkd_resume_host(self.algo, current & 0xFFFFFFFF, ptr, length, ctypes.byref(out)))
            del view
        return to_java_int(out.value)

    # IntHash.acceptsMemoryAddressBuffer (IntHash.java:34; JniIntHash.java:60-63)
    def acceptsMemoryAddressBuffer(self) -> bool:
        return True

    # ---- batch extension (the reference has none) ----
    def resumeBatch(self, seeds, base, offsets, lengths, out=None, stream=None):
        return crc_batch(self.algo, base, offsets, lengths, seeds=seeds, out=out, stream=stream)


class Crc32cIntChecksum:
    """Static facade (Crc32cIntChecksum.java:24-100). The reference selects its provider once at class
    init and never throws (:28-36); here the one provider is libbkdigest.so, whose host-buffer resume
    has its own CPU route, so a missing GPU is not an error. A missing library is (NativeUnavailable):
    it is the product, and nothing here substitutes Python arithmetic for it."""

    _hash: GpuIntHash | None = None

    @classmethod
    def _h(cls) -> GpuIntHash:
        if cls._hash is None:
            cls._hash = GpuIntHash(CRC32C)
        return cls._hash

    @classmethod
    def computeChecksum(cls, payload, offset: int | None = None, length: int | None = None) -> int:
        return cls._h().calculate(payload, offset, length)

    @classmethod
    def resumeChecksum(cls, previousChecksum: int, payload, offset: int | None = None,
                       length: int | None = None) -> int:
        return cls._h().resume(previousChecksum, payload, offset, length)

    @classmethod
    def acceptsMemoryAddressBuffer(cls) -> bool:
        return cls._h().acceptsMemoryAddressBuffer()


# ---------------------------------------------------------------------------------------------
# Device-resident batch API (torch tensors on a HIP device)
# ---------------------------------------------------------------------------------------------

def _dev_ptr(t, name: str, dtype=None, device=None, min_numel: int | None = None):
    """Device pointer of a contiguous tensor, checked: on `device` (the base buffer's), of `dtype`
    (a dtype or a tuple of allowed dtypes) and with at least `min_numel` elements."""
    if t is None:
        return ctypes.c_void_p(0)
    if not (_is_torch_tensor(t) and t.is_cuda):
        raise TypeError(f"{name} must be a torch tensor on a HIP device")
    if dtype is not None:
        allowed = dtype if isinstance(dtype, tuple) else (dtype,)
        if t.dtype not in allowed:
            raise TypeError(f"{name} must have dtype {' or '.join(str(d) for d in allowed)}, not {t.dtype}")
    if device is not None and t.device != device:
        raise ValueError(f"{name} is on {t.device} but the base buffer is on {device}")
    if min_numel is not None and t.numel() < min_numel:
        raise ValueError(f"{name} has {t.numel()} elements, needs {min_numel}")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return ctypes.c_void_p(t.data_ptr())


def _u32_dtypes():
    import torch
    return (torch.int32, torch.uint32) if hasattr(torch, "uint32") else (torch.int32,)


def crc_batch_uniform(algo: int, base, entry_len: int, n: int, stride: int | None = None, seeds=None,
                      seed_all: int = 0, out=None, stream=None):
    """out[i] = resume(seed_i, base[i*stride : i*stride + entry_len]) on the device."""
    import torch
    stride = entry_len if stride is None else stride
    nbytes = base.numel() * base.element_size()
    if n and (n - 1) * stride + entry_len > nbytes:
        raise IndexError("uniform batch exceeds base buffer")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    u32, dev = _u32_dtypes(), base.device
    with _on_device(base):
        check(lib().bkd_crc_batch_uniform(algo, _dev_ptr(base, "base"), stride, entry_len, n,
                                          _dev_ptr(seeds, "seeds", u32, dev, n), seed_all & 0xFFFFFFFF,
                                          _dev_ptr(out, "out", u32, dev, n), _stream_ptr(stream, base)))
    return out


def crc_batch(algo: int, base, offsets, lengths, seeds=None, seed_all: int = 0, out=None, stream=None,
              sync_check: bool = False):
    """out[i] = resume(seed_i, base[offsets[i] : offsets[i] + lengths[i]]) on the device.

    offsets: int64 tensor, lengths: int32 tensor (values < 2^32), seeds: int32 tensor or None.
    Out-of-range entries produce 0 and make ``bkd_stream_sync`` report BKD_ERR_BOUNDS
    (checked here when ``sync_check``)."""
    import torch
    n = offsets.numel()
    if lengths.numel() != n:
        raise ValueError("offsets/lengths size mismatch")
    if out is None:
        out = torch.empty(n, dtype=torch.int32, device=base.device)
    nbytes = base.numel() * base.element_size()
    u32, dev = _u32_dtypes(), base.device
    with _on_device(base):
        st = _stream_ptr(stream, base)
        check(lib().bkd_crc_batch(algo, _dev_ptr(base, "base"), nbytes, _dev_ptr(offsets, "offsets", torch.int64, dev),
                                  _dev_ptr(lengths, "lengths", u32, dev), n, _dev_ptr(seeds, "seeds", u32, dev, n),
                                  seed_all & 0xFFFFFFFF, _dev_ptr(out, "out", u32, dev, n), st))
        if sync_check:
            check(lib().bkd_stream_sync(st))
    return out


def crc_batch_segments(algo: int, base, seg_offsets, seg_lengths, seg_first, seeds=None, seed_all: int = 0,
                       out=None, stream=None, sync_check: bool = False):
    """Composite entries (bkd_crc_batch_segments): out[i] = resume(seed_i, the concatenation of
    segments seg_first[i] .. seg_first[i+1]-1), segment k = base[seg_offsets[k] : + seg_lengths[k]].

    seg_offsets: int64, seg_lengths: int32, seg_first: int64 with n + 1 entries (torch, on the device)."""
    import torch
    nseg = seg_offsets.numel()
    n = seg_first.numel() - 1
    if n < 0:
        raise ValueError("seg_first needs n + 1 entries")
    if seg_lengths.numel() != nseg:
        raise ValueError("seg_offsets/seg_lengths size mismatch")
    if out is None:
        out = torch.empty(max(n, 0), dtype=torch.int32, device=base.device)
    u32, dev = _u32_dtypes(), base.device
    with _on_device(base):
        st = _stream_ptr(stream, base)
        check(lib().bkd_crc_batch_segments(algo, _dev_ptr(base, "base"), base.numel() * base.element_size(),
                                           _dev_ptr(seg_offsets, "seg_offsets", torch.int64, dev),
                                           _dev_ptr(seg_lengths, "seg_lengths", u32, dev), nseg,
                                           _dev_ptr(seg_first, "seg_first", torch.int64, dev), n,
                                           _dev_ptr(seeds, "seeds", u32, dev, n), seed_all & 0xFFFFFFFF,
                                           _dev_ptr(out, "out", u32, dev, n), st))
        if sync_check:
            check(lib().bkd_stream_sync(st))
    return out


def crc_batch_host(algo: int, base, offsets, lengths, seeds=None, seed_all: int = 0) -> np.ndarray:
    """Host-memory batch; returns uint32 CRCs. Route (set_host_batch_route): the GPU (H2D -> kernel
    -> D2H inside the library) or the library's threaded CPU route."""
    view = _host_view(base)
    offsets = np.ascontiguousarray(offsets, dtype=np.uint64)
    lengths = np.ascontiguousarray(lengths, dtype=np.uint32)
    n = offsets.size
    if lengths.size != n:
        raise ValueError("offsets/lengths size mismatch")
    out = np.zeros(n, dtype=np.uint32)
    sp = ctypes.c_void_p(0)
    if seeds is not None:
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        if seeds.size < n:
            raise ValueError(f"seeds has {seeds.size} elements, needs {n}")
        sp = ctypes.c_void_p(seeds.ctypes.data)
    check(lib().bkd_crc_batch_host(algo, ctypes.c_void_p(view.ctypes.data if view.size else 0), view.size,
                                   ctypes.c_void_p(offsets.ctypes.data), ctypes.c_void_p(lengths.ctypes.data), n,
                                   sp, seed_all & 0xFFFFFFFF, ctypes.c_void_p(out.ctypes.data)))
    return out


def fill_splitmix64(buf, seed: int, first_word: int = 0, stream=None) -> None:
    """Device-side synthetic input: little-endian splitmix64 words."""
    nbytes = buf.numel() * buf.element_size()
    with _on_device(buf):
        check(lib().bkd_fill_splitmix64(_dev_ptr(buf, "buf"), nbytes, seed & (2**64 - 1), first_word,
                                        _stream_ptr(stream, buf)))


def stream_sync(stream) -> None:
    """Waits for `stream` and raises BKD_ERR_BOUNDS if an indexed batch enqueued on it since its
    previous sync had an entry outside its base buffer (bkd_stream_sync; the flag is per stream)."""
    ptr = _stream_ptr(stream)
    sdev = getattr(stream, "device", None)
    if sdev is not None:
        import torch
        with torch.cuda.device(sdev):
            check(lib().bkd_stream_sync(ptr))
    else:
        check(lib().bkd_stream_sync(ptr))


def release_stream(stream) -> None:
    """Waits for `stream` and frees the library's scratch for it (bkd_stream_release): call before a
    stream that ran indexed batches is dropped. Raises BKD_ERR_BOUNDS as a sync would."""
    ptr = _stream_ptr(stream)
    sdev = getattr(stream, "device", None)
    if sdev is not None:
        import torch
        with torch.cuda.device(sdev):
            check(lib().bkd_stream_release(ptr))
    else:
        check(lib().bkd_stream_release(ptr))


def cpu_resume(algo: int, current: int, buffer) -> int:
    """The library's CPU route only (bkd_cpu_resume), whatever the size; Java int bit pattern."""
    view = _host_view(buffer)
    out = ctypes.c_uint32(0)
    check(lib().bkd_cpu_resume(algo, current & 0xFFFFFFFF, ctypes.c_void_p(view.ctypes.data if view.size else 0),
                               view.size, ctypes.byref(out)))
    return to_java_int(out.value)


HOST_ROUTE_AUTO, HOST_ROUTE_CPU, HOST_ROUTE_GPU = 0, 1, 2
_host_route = HOST_ROUTE_AUTO  # the route last set through this module


def set_host_batch_route(route: int) -> None:
    """Route of host-resident batches: 0 auto (measured crossover), 1 CPU threads, 2 GPU."""
    global _host_route
    check(lib().bkd_set_host_batch_route(route))
    _host_route = route


def get_host_batch_route() -> int:
    """The route the next host-resident batch takes: 1 CPU, 2 GPU."""
    return int(lib().bkd_get_host_batch_route())


@contextlib.contextmanager
def host_batch_route(route: int):
    """Temporarily force the host-resident batch route (tests, benchmarks); restores the previous one."""
    prev = _host_route
    set_host_batch_route(route)
    try:
        yield
    finally:
        set_host_batch_route(prev)


def set_host_threads(threads: int) -> None:
    """Host threads the CPU route and staging copies may use (0 = the whole pool)."""
    check(lib().bkd_set_host_threads(threads))


def get_host_threads() -> int:
    return int(lib().bkd_get_host_threads())


def host_release() -> None:
    """Frees the idle pinned staging sets of the host batches' GPU route (bkd_host_release)."""
    check(lib().bkd_host_release())


def set_cpu_route_max(nbytes: int) -> None:
    """Host buffers up to nbytes take the CPU route in per-call resumes (0 = GPU whenever present)."""
    check(lib().bkd_set_cpu_route_max(nbytes))


def get_cpu_route_max() -> int:
    return int(lib().bkd_get_cpu_route_max())


def cpu_impl() -> str:
    return lib().bkd_cpu_impl().decode()


def set_group_lanes(lanes: int) -> None:
    check(lib().bkd_set_group_lanes(lanes))


def set_fold_schedule(schedule: int) -> None:
    """0 = by the measured shader clock (default), 1 = compiler schedule, 2 = low-clock schedule."""
    check(lib().bkd_set_fold_schedule(schedule))


def set_plan_mode(mode: int) -> None:
    """0 = auto, 1 = one entry per lane group, 2 = chunked plan (indexed batches)."""
    check(lib().bkd_set_plan_mode(mode))


def set_plan_small(max_bytes: int = 192) -> None:
    """Entries of <= max_bytes (<= 512) of a planned indexed batch run in the short-entry launch (0 = none)."""
    check(lib().bkd_set_plan_small(max_bytes))


def set_short_class_mean(max_bytes_per_entry: int) -> None:
    """The short-entry class runs when the base buffer holds at most this many bytes per entry
    (default 1024; 2**64 - 1: whenever a bound is set)."""
    check(lib().bkd_set_short_class_mean(max_bytes_per_entry))


def set_plan_serial(max_bytes: int = 16) -> None:
    """Plan entries shorter than max_bytes (16..64) are computed by the combine kernel, one thread each."""
    check(lib().bkd_set_plan_serial(max_bytes))


def set_plan_prefetch(loads_in_flight: int = 2) -> None:
    check(lib().bkd_set_plan_prefetch(loads_in_flight))


def set_plan_geometry(lanes: int = 8, steps_per_chunk: int = 32, merge_bytes: int = 16) -> None:
    check(lib().bkd_set_plan_geometry(lanes, steps_per_chunk, merge_bytes))


def host_tables(algo: int, lanes: int) -> np.ndarray:
    # operator sets, byte table, x^64 / x^96 sets, and for 4 / 8 lanes the lane-position nibble tables
    n = (2 + int(np.log2(lanes))) * 1024 + 256 + 2048 + (128 * lanes if lanes in (4, 8) else 0)
    out = np.zeros(n, dtype=np.uint32)
    check(lib().bkd_host_tables(algo, lanes, ctypes.c_void_p(out.ctypes.data), n))
    return out


device_count = _native.device_count
