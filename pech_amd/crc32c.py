"""Python mirror of the C-ABI (include/crc32c.h, include/pech_crc32c.h).

Same names and argument meaning as the reference's crc32c()
(/root/reference/include/crc32c.h:88): `crc` is the incoming raw register,
the result is the raw register after the bytes, no inversion.  Device
buffers are torch uint8 tensors on a ROCm device (torch is plumbing here:
device memory and streams); every checksum is computed by the gfx950 kernel
in libpech_crc32c.so, except the drop-in crc32c()'s small calls, which the
library computes on the host as SURVEY.md §8(a) a7/a8 prescribe (see
set_cpu_max / stats).
"""
import ctypes

import numpy as np

from ._lib import CDesc, Crc32cError, check, lib

__all__ = [
    "crc32c", "crc32c_batch", "crc32c_shift", "crc32c_combine", "make_descs", "dev_batch_async",
    "dev_batch_small_async", "dev_batch_ws_async", "dev_copy_batch_ws_async", "workspace_bytes", "crc32c_tensors", "shard_ranges", "Crc32cError", "timing",
    "timing_read", "timing_samples", "version", "crc32c_concat", "Pages", "AsyncCrc", "async_devices", "set_cpu_max", "set_flat_max", "stats",
]

F_HOST, F_DEVICE, F_PINNED, F_ALL_DEVICES = 0, 1, 2, 4


def crc32c(crc, data):
    """crc32c(crc, data) over host bytes (include/crc32c.h:88 semantics)."""
    mv = memoryview(data).cast("B")
    n = mv.nbytes
    if n == 0:
        return crc & 0xFFFFFFFF
    buf = (ctypes.c_char * n).from_buffer_copy(mv) if mv.readonly else (ctypes.c_char * n).from_buffer(mv)
    return lib().crc32c(crc & 0xFFFFFFFF, ctypes.addressof(buf), n)


def set_cpu_max(nbytes):
    """Drop-in routing: crc32c() calls of at most nbytes run on the host CPU
    (0: every non-empty call on the GPU).  Returns the previous value."""
    return int(lib().crc32c_set_cpu_max(int(nbytes)))


def set_flat_max(n):
    """Device batches of at most n buffers run as one launch with no plan
    kernel (pech_crc32c_flat up to 256, pech_crc32c_flatg up to 4,096;
    default and maximum 4,096, 0 = always plan + main).  Returns the previous value (0 from a pre-flat release loaded
    for an A/B, which always plans)."""
    fn = getattr(lib(), "crc32c_set_flat_max", None)
    return int(fn(int(n))) if fn is not None else 0


def stats():
    """The drop-in's process-wide counters (struct crc32c_stats) as a dict."""
    from ._lib import CStats

    st = CStats()
    check(lib().crc32c_get_stats(ctypes.byref(st)), "crc32c_get_stats")
    return {name: int(getattr(st, name)) for name, _ in CStats._fields_}


def crc32c_batch(bufs, seeds=None):
    """One independent CRC per host buffer (bytes-like), as a list of ints."""
    n = len(bufs)
    if n == 0:
        return []
    keep = []
    ptrs = (ctypes.c_void_p * n)()
    lens = (ctypes.c_uint * n)()
    for i, b in enumerate(bufs):
        mv = memoryview(b).cast("B")
        c = (ctypes.c_char * max(mv.nbytes, 1)).from_buffer_copy(mv.tobytes() or b"\0")
        keep.append(c)
        ptrs[i] = ctypes.addressof(c)
        lens[i] = mv.nbytes
    sd = None
    if seeds is not None:
        sd = (ctypes.c_uint32 * n)(*[s & 0xFFFFFFFF for s in seeds])
    out = (ctypes.c_uint32 * n)()
    check(lib().crc32c_batch(ptrs, lens, sd, out, n, F_HOST), "crc32c_batch")
    return list(out)


def crc32c_shift(v, nbytes):
    return lib().crc32c_shift(v & 0xFFFFFFFF, nbytes)


def crc32c_combine(crc_a, crc_b, len_b):
    return lib().crc32c_combine(crc_a & 0xFFFFFFFF, crc_b & 0xFFFFFFFF, len_b)


def make_descs(addrs, lens, seeds=None, device=None):
    """Pack descriptors (struct crc32c_desc, 16 B each) into an int64 tensor
    of shape (n, 2): [addr, len | seed << 32]; on `device` if given."""
    import torch

    addrs = np.asarray(addrs, dtype=np.uint64)
    lens = np.asarray(lens, dtype=np.uint64)
    seeds = np.zeros_like(lens) if seeds is None else np.asarray(seeds, dtype=np.uint64) & np.uint64(0xFFFFFFFF)
    if np.any(lens > np.uint64(0xFFFFFFFF)):
        raise ValueError("buffer length must fit unsigned int (crc32c.h:88)")
    packed = np.empty((len(addrs), 2), dtype=np.uint64)
    packed[:, 0] = addrs
    packed[:, 1] = lens | (seeds << np.uint64(32))
    t = torch.from_numpy(packed.view(np.int64).copy())
    return t.to(device) if device is not None else t


def dev_batch_async(descs, out, stream=None):
    """Enqueue the device batch: descs (n,2) int64 device tensor from
    make_descs, out (n,) int32/uint32 device tensor.  `stream` is a
    torch.cuda.Stream (default: torch's current stream)."""
    import torch

    n = descs.shape[0]
    if out.numel() < n or out.element_size() != 4:
        raise ValueError("out must hold n 32-bit words")
    if stream is None:
        stream = torch.cuda.current_stream(descs.device)
    check(lib().crc32c_dev_batch_async(descs.data_ptr(), out.data_ptr(), n, stream.cuda_stream),
          "crc32c_dev_batch_async")


def dev_batch_small_async(descs, out, stream=None):
    """The small-buffer device batch (crc32c_dev_batch_small_async): one
    launch, no workspace, graph-capturable; balanced for buffers below
    32 KiB, correct for any."""
    import torch

    n = descs.shape[0]
    if out.numel() < n or out.element_size() != 4:
        raise ValueError("out must hold n 32-bit words")
    if stream is None:
        stream = torch.cuda.current_stream(descs.device)
    check(lib().crc32c_dev_batch_small_async(descs.data_ptr(), out.data_ptr(), n, stream.cuda_stream),
          "crc32c_dev_batch_small_async")


def workspace_bytes(n):
    """Device workspace one launch of n buffers needs (crc32c_dev_workspace_bytes)."""
    return int(lib().crc32c_dev_workspace_bytes(n))


def dev_batch_ws_async(descs, out, ws, stream=None):
    """dev_batch_async with an explicit workspace (uint8 device tensor of at
    least workspace_bytes(n), 256-byte aligned): one workspace per stream
    lets independent batches run concurrently on several streams."""
    import torch

    n = descs.shape[0]
    if out.numel() < n or out.element_size() != 4:
        raise ValueError("out must hold n 32-bit words")
    if stream is None:
        stream = torch.cuda.current_stream(descs.device)
    check(lib().crc32c_dev_batch_ws_async(descs.data_ptr(), out.data_ptr(), n, ws.data_ptr(), ws.numel(),
                                          stream.cuda_stream), "crc32c_dev_batch_ws_async")


def dev_copy_batch_ws_async(descs, dsts, out, ws, stream=None):
    """Fused CRC + copy (crc32c_dev_copy_batch_ws_async): dsts is an (n,)
    int64 device tensor of destination addresses."""
    import torch

    n = descs.shape[0]
    if out.numel() < n or out.element_size() != 4 or dsts.numel() < n or dsts.element_size() != 8:
        raise ValueError("out must hold n 32-bit words, dsts n 64-bit addresses")
    if stream is None:
        stream = torch.cuda.current_stream(descs.device)
    check(lib().crc32c_dev_copy_batch_ws_async(descs.data_ptr(), dsts.data_ptr(), out.data_ptr(), n, ws.data_ptr(),
                                               ws.numel(), stream.cuda_stream), "crc32c_dev_copy_batch_ws_async")


def dev_copy_batch_small_async(descs, dsts, out, stream=None):
    """Fused CRC + copy of a small-buffer batch (crc32c_dev_copy_batch_small_async):
    one launch of the direct kernel, no workspace; balanced for buffers below
    32 KiB, correct for any."""
    import torch

    n = descs.shape[0]
    if out.numel() < n or out.element_size() != 4 or dsts.numel() < n or dsts.element_size() != 8:
        raise ValueError("out must hold n 32-bit words, dsts n 64-bit addresses")
    if stream is None:
        stream = torch.cuda.current_stream(descs.device)
    check(lib().crc32c_dev_copy_batch_small_async(descs.data_ptr(), dsts.data_ptr(), out.data_ptr(), n,
                                                  stream.cuda_stream), "crc32c_dev_copy_batch_small_async")


def crc32c_tensors(tensors, seeds=None, offsets=None, lengths=None):
    """CRCs of device uint8 tensors (optionally sub-ranges [off, off+len)).
    Synchronous convenience wrapper; returns a list of ints."""
    import torch

    n = len(tensors)
    if n == 0:
        return []
    dev = tensors[0].device
    addrs = [t.data_ptr() + (offsets[i] if offsets else 0) for i, t in enumerate(tensors)]
    lens = [lengths[i] if lengths else t.numel() * t.element_size() for i, t in enumerate(tensors)]
    descs = make_descs(addrs, lens, seeds, device=dev)
    out = torch.empty(n, dtype=torch.int32, device=dev)
    with torch.cuda.device(dev):
        dev_batch_async(descs, out)
        torch.cuda.current_stream(dev).synchronize()
    return [int(x) & 0xFFFFFFFF for x in out.cpu().numpy().view(np.uint32)]


def shard_ranges(lens, world):
    """Contiguous, byte-balanced split of a batch over `world` GPUs
    (greedy prefix split of sum(len)).  Returns [(lo, hi)]
    index ranges covering [0, n) in order; empty ranges allowed."""
    lens = np.asarray(lens, dtype=np.float64)
    n = len(lens)
    if world <= 0:
        raise ValueError("world must be positive")
    csum = np.concatenate([[0.0], np.cumsum(lens)])
    total = csum[-1]
    cuts = [0]
    for r in range(1, world):
        target = total * r / world
        cut = int(np.searchsorted(csum, target, side="left"))
        cuts.append(min(max(cut, cuts[-1]), n))
    cuts.append(n)
    return [(cuts[r], cuts[r + 1]) for r in range(world)]


def timing(enable=True):
    check(lib().crc32c_timing(1 if enable else 0), "crc32c_timing")


def timing_read():
    """(kernel_ms, launches) of main-kernel launches since the last read."""
    ms = ctypes.c_double()
    cnt = ctypes.c_uint64()
    check(lib().crc32c_timing_read(ctypes.byref(ms), ctypes.byref(cnt)), "crc32c_timing_read")
    return ms.value, cnt.value


def timing_samples():
    """Per-launch main-kernel milliseconds gathered by the last timing_read()."""
    n = lib().crc32c_timing_samples(None, 0)
    buf = (ctypes.c_float * max(n, 1))()
    lib().crc32c_timing_samples(buf, n)
    return list(buf)[:n]


def version():
    return lib().crc32c_version().decode()


def crc32c_concat(seed, crcs, lens):
    """crc32c(seed, S_0 || ... || S_n-1) from zero-seeded segment CRCs
    (include/pech_crc32c_async.h; host algebra, no data pass)."""
    n = len(crcs)
    c = (ctypes.c_uint32 * max(n, 1))(*[int(x) & 0xFFFFFFFF for x in crcs])
    l = (ctypes.c_uint64 * max(n, 1))(*[int(x) for x in lens])
    return lib().crc32c_concat(seed & 0xFFFFFFFF, c, l, n)


class Pages:
    """crc32c_pages_alloc(order) memory (pinned, GPU-mapped host pages) as a
    writable numpy uint8 view; free() returns it to the per-order cache."""

    def __init__(self, order):
        self.order = order
        self.nbytes = 4096 << order
        self.ptr = lib().crc32c_pages_alloc(order)
        if not self.ptr:
            raise Crc32cError(f"crc32c_pages_alloc({order}) failed: {lib().crc32c_last_error().decode()}")
        self.view = np.ctypeslib.as_array((ctypes.c_uint8 * self.nbytes).from_address(self.ptr))

    def free(self):
        if self.ptr:
            lib().crc32c_pages_free(self.ptr, self.order)
            self.ptr = None
            self.view = None


def async_devices():
    """crc32c_async_devices: the GPUs to spread async contexts over (every
    visible device, or the PECH_DEVICES list)."""
    devs = (ctypes.c_int * 64)()
    n = lib().crc32c_async_devices(devs, 64)
    check(n if n < 0 else 0, "crc32c_async_devices")
    return list(devs[:n])


class AsyncCrc:
    """crc32c_async context (include/pech_crc32c_async.h): submit host
    payloads, poll fd() from an event loop, complete() runs the callbacks."""

    def __init__(self, dma=False, zerocopy=None, device=None):
        """dma=False: crc32c_pages payloads are read in place (the default);
        dma=True: CRC32C_ASYNC_DMA, DMA'd to device staging at launch.
        zerocopy: the round-3 keyword, kept as an alias (zerocopy=True is the
        default mode, CRC32C_ASYNC_ZEROCOPY; zerocopy=False asks for DMA);
        zerocopy=True together with dma=True is refused, as
        crc32c_async_create refuses both flags.  device: the GPU
        (crc32c_async_create_on), default the current one."""
        from ._lib import DONE_FN

        if zerocopy is not None:
            if zerocopy and dma:
                raise ValueError("AsyncCrc: zerocopy=True and dma=True are exclusive")
            dma = dma or not zerocopy
        flags = 2 if dma else (1 if zerocopy else 0)
        self._h = lib().crc32c_async_create(flags) if device is None else lib().crc32c_async_create_on(device, flags)
        if not self._h:
            raise Crc32cError(f"crc32c_async_create failed: {lib().crc32c_last_error().decode()}")
        self._keep = {}  # submission key -> (payload ref, python callback)
        self._next = 0
        self.stray = 0  # callbacks for submissions that returned an error (must stay 0)

        def trampoline(arg, crc, err):
            ent = self._keep.pop(arg, None)
            if ent is None:
                self.stray += 1
                return
            ent[1](crc, err)

        self._cfn = DONE_FN(trampoline)

    @property
    def handle(self):
        return self._h

    def stats(self):
        """crc32c_async_get_stats as a dict (device, submitted, launches,
        inflight, queued, host_out, polled)."""
        from ._lib import CAsyncStats

        st = CAsyncStats()
        check(lib().crc32c_async_get_stats(self._h, ctypes.byref(st)), "crc32c_async_get_stats")
        return {name: int(getattr(st, name)) for name, _ in CAsyncStats._fields_}

    def fd(self):
        return lib().crc32c_async_fd(self._h)

    def submit(self, buf, length, seed, callback, keep=None):
        """buf: integer address of host bytes; callback(crc, err)."""
        self._next += 1
        key = self._next
        self._keep[key] = (keep, callback)
        rc = lib().crc32c_async_submit(self._h, buf, length, seed & 0xFFFFFFFF, self._cfn, key)
        if rc:
            self._keep.pop(key, None)
            check(rc, "crc32c_async_submit")

    def flush(self):
        check(lib().crc32c_async_flush(self._h), "crc32c_async_flush")

    def complete(self):
        rc = lib().crc32c_async_complete(self._h)
        if rc < 0:
            check(rc, "crc32c_async_complete")
        return rc

    def drain(self):
        check(lib().crc32c_async_drain(self._h), "crc32c_async_drain")

    def pending(self):
        return lib().crc32c_async_pending(self._h)

    def close(self):
        if self._h:
            lib().crc32c_async_destroy(self._h)
            self._h = None
