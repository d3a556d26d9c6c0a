"""ctypes binding of libpech_crc32c.so (the C-ABI in include/*.h).

The library is built in-tree by `make` (__graft_entry__.build()).  There is
no fallback: if the shared library is missing or a symbol is absent, loading
raises, and compute calls report the library's own error text.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
# PECH_CRC32C_LIB selects an alternative build (A/B experiments only)
LIB_PATH = os.environ.get("PECH_CRC32C_LIB") or os.path.join(HERE, "libpech_crc32c.so")

_lib = None


class Crc32cError(RuntimeError):
    pass


class CDesc(ctypes.Structure):
    """struct crc32c_desc (include/pech_crc32c.h)."""
    _fields_ = [("addr", ctypes.c_uint64), ("len", ctypes.c_uint32), ("seed", ctypes.c_uint32)]


class CStats(ctypes.Structure):
    """struct crc32c_stats (include/pech_crc32c.h)."""
    _fields_ = [("cpu_calls", ctypes.c_uint64), ("cpu_bytes", ctypes.c_uint64), ("gpu_calls", ctypes.c_uint64),
                ("gpu_bytes", ctypes.c_uint64), ("gpu_fallbacks", ctypes.c_uint64), ("gpu_faults", ctypes.c_uint64)]


class CAsyncStats(ctypes.Structure):
    """struct crc32c_async_stats (include/pech_crc32c_async.h)."""
    _fields_ = [("device", ctypes.c_int), ("submitted", ctypes.c_uint64), ("launches", ctypes.c_uint64),
                ("inflight", ctypes.c_uint), ("queued", ctypes.c_uint), ("host_out", ctypes.c_uint64),
                ("polled", ctypes.c_uint64), ("faults", ctypes.c_uint64), ("pub_missing", ctypes.c_uint64)]


# completion callback of include/pech_crc32c_async.h: (arg, crc, err)
DONE_FN = ctypes.CFUNCTYPE(None, ctypes.c_void_p, ctypes.c_uint32, ctypes.c_int)

# name -> (restype, argtypes); must cover every function in include/*.h
SIGNATURES = {
    "crc32c": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint]),
    "crc32c_batch": (ctypes.c_int, [ctypes.POINTER(ctypes.c_void_p), ctypes.POINTER(ctypes.c_uint),
                                     ctypes.POINTER(ctypes.c_uint32), ctypes.POINTER(ctypes.c_uint32),
                                     ctypes.c_uint, ctypes.c_uint]),
    "crc32c_dev_batch_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]),
    "crc32c_dev_batch_small_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                                    ctypes.c_void_p]),
    "crc32c_dev_workspace_bytes": (ctypes.c_size_t, [ctypes.c_uint]),
    "crc32c_dev_batch_ws_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p,
                                                 ctypes.c_size_t, ctypes.c_void_p]),
    "crc32c_dev_reserve": (ctypes.c_int, [ctypes.c_uint]),
    "crc32c_dev_copy_batch_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                                   ctypes.c_void_p]),
    "crc32c_dev_copy_batch_ws_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                      ctypes.c_uint, ctypes.c_void_p, ctypes.c_size_t,
                                                      ctypes.c_void_p]),
    "crc32c_dev_copy_batch_small_async": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                                         ctypes.c_uint, ctypes.c_void_p]),
    "crc32c_shift": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint64]),
    "crc32c_combine": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]),
    "crc32c_device_init": (ctypes.c_int, []),
    "crc32c_set_cpu_max": (ctypes.c_uint, [ctypes.c_uint]),
    "crc32c_set_flat_max": (ctypes.c_uint, [ctypes.c_uint]),
    "crc32c_get_stats": (ctypes.c_int, [ctypes.c_void_p]),
    "crc32c_timing": (ctypes.c_int, [ctypes.c_int]),
    "crc32c_timing_read": (ctypes.c_int, [ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_uint64)]),
    "crc32c_timing_samples": (ctypes.c_int, [ctypes.POINTER(ctypes.c_float), ctypes.c_uint]),
    "crc32c_last_error": (ctypes.c_char_p, []),
    # include/pech_crc32c_async.h
    "crc32c_pages_alloc": (ctypes.c_void_p, [ctypes.c_uint]),
    "crc32c_pages_free": (None, [ctypes.c_void_p, ctypes.c_uint]),
    "crc32c_pages_is_pinned": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_size_t]),
    "crc32c_pages_trim": (None, []),
    "crc32c_async_create": (ctypes.c_void_p, [ctypes.c_uint]),
    "crc32c_async_create_on": (ctypes.c_void_p, [ctypes.c_int, ctypes.c_uint]),
    "crc32c_msgr_conn_async": (ctypes.c_void_p, [ctypes.c_void_p]),
    "crc32c_async_devices": (ctypes.c_int, [ctypes.POINTER(ctypes.c_int), ctypes.c_int]),
    "crc32c_async_get_stats": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "crc32c_async_fd": (ctypes.c_int, [ctypes.c_void_p]),
    "crc32c_async_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint, ctypes.c_uint32,
                                           DONE_FN, ctypes.c_void_p]),
    "crc32c_async_flush": (ctypes.c_int, [ctypes.c_void_p]),
    "crc32c_async_complete": (ctypes.c_int, [ctypes.c_void_p]),
    "crc32c_async_drain": (ctypes.c_int, [ctypes.c_void_p]),
    "crc32c_async_pending": (ctypes.c_uint, [ctypes.c_void_p]),
    "crc32c_async_destroy": (None, [ctypes.c_void_p]),
    "crc32c_concat": (ctypes.c_uint32, [ctypes.c_uint32, ctypes.POINTER(ctypes.c_uint32),
                                        ctypes.POINTER(ctypes.c_uint64), ctypes.c_uint]),
    "crc32c_version": (ctypes.c_char_p, []),
    # include/pech_crc32c_msgr.h (callbacks as plain pointers: driven from C, tests/c/msgr_conn_sim.c)
    "crc32c_msgr_conn_create": (ctypes.c_void_p, [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p, ctypes.c_void_p,
                                                 ctypes.c_void_p]),
    "crc32c_msgr_conn_reset": (None, [ctypes.c_void_p]),
    "crc32c_msgr_conn_destroy": (None, [ctypes.c_void_p]),
    "crc32c_msgr_rx_queue": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                            ctypes.c_int, ctypes.c_uint32]),
    "crc32c_msgr_rx_next": (ctypes.c_int, [ctypes.c_void_p, ctypes.POINTER(ctypes.c_void_p),
                                           ctypes.POINTER(ctypes.c_uint32)]),
    "crc32c_msgr_rx_pending": (ctypes.c_uint, [ctypes.c_void_p]),
    "crc32c_msgr_tx_submit": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint,
                                             ctypes.c_uint32]),
    "crc32c_msgr_tx_known": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_uint32]),
    "crc32c_msgr_tx_footer": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p, ctypes.POINTER(ctypes.c_uint32)]),
    "crc32c_msgr_get_stats": (None, [ctypes.c_void_p]),
    "crc32c_msgr_set_host_max": (ctypes.c_uint, [ctypes.c_uint]),
    "crc32c_msgr_set_lone_max": (ctypes.c_uint, [ctypes.c_uint]),
    "crc32c_msgr_tx_has": (ctypes.c_int, [ctypes.c_void_p, ctypes.c_void_p]),
    "crc32c_msgr_tx_cancel": (ctypes.c_uint, [ctypes.c_void_p, ctypes.c_void_p]),
}


class CMsgrStats(ctypes.Structure):
    """struct crc32c_msgr_stats (include/pech_crc32c_msgr.h)."""
    _fields_ = [(n, ctypes.c_uint64) for n in ("rx_submitted", "rx_unchecked", "rx_verified", "rx_bad",
                                                "rx_released", "tx_submitted", "tx_known", "tx_held",
                                                "tx_released", "rx_host", "tx_host", "rx_lone", "tx_lone")]


def lib():
    """Load (once) and return the C library; raises if it is not built."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise Crc32cError(f"{LIB_PATH} is missing: run `make` (or __graft_entry__.build()) first")
        L = ctypes.CDLL(LIB_PATH)
        for name, (res, args) in SIGNATURES.items():
            # an older release loaded for a same-box A/B (PECH_CRC32C_LIB) may
            # lack later entry points; the current library exports all of
            # them (tests/test_abi.py)
            fn = getattr(L, name, None)
            if fn is None and "PECH_CRC32C_LIB" in os.environ:
                continue
            if fn is None:
                raise Crc32cError(f"{LIB_PATH} does not export {name}")
            fn.restype = res
            fn.argtypes = args
        _lib = L
    return _lib


def check(rc, what):
    if rc != 0:
        err = lib().crc32c_last_error().decode(errors="replace")
        raise Crc32cError(f"{what} failed ({rc}): {err}")
    return rc
