"""Test-side access to the oracle (oracle/liboracle_crc32c.so, the C
restatement) and, when built, to oracle/_ref/libref_crc32c.so (the
reference header compiled from /root/reference).  Test infrastructure only.
"""
import ctypes
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_SO = os.path.join(REPO, "oracle", "liboracle_crc32c.so")
REF_SO = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")
HW_SO = os.path.join(REPO, "oracle", "liboracle_hw.so")

_o = None
_r = None
_h = None


def hw():
    """SSE4.2 CRC32C (oracle/crc32c_hw.c): a CPU context baseline, or None
    when the library is absent or this host lacks SSE4.2."""
    global _h
    if _h is None:
        try:
            flags = open("/proc/cpuinfo").read()
        except OSError:
            flags = ""
        if " sse4_2" not in flags:
            return None
        if not os.path.exists(HW_SO):
            subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "all"])
        L = ctypes.CDLL(HW_SO)
        L.hw_crc32c.restype = ctypes.c_uint32
        L.hw_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint]
        L.hw_crc32c_batch_mt.restype = ctypes.c_int
        L.hw_crc32c_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                         ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
        _h = L
    return _h


def oracle():
    global _o
    if _o is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.check_call(["make", "-C", os.path.join(REPO, "oracle"), "all"])
        L = ctypes.CDLL(ORACLE_SO)
        L.oracle_crc32c.restype = ctypes.c_uint32
        L.oracle_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint]
        L.oracle_crc32c_batch.restype = None
        L.oracle_crc32c_batch.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                          ctypes.c_uint]
        L.oracle_crc32c_strided.restype = None
        L.oracle_crc32c_strided.argtypes = [ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint, ctypes.c_void_p,
                                            ctypes.c_uint]
        L.oracle_crc32c_pieces.restype = ctypes.c_uint32
        L.oracle_crc32c_pieces.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_uint]
        L.oracle_shift.restype = ctypes.c_uint32
        L.oracle_shift.argtypes = [ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_combine.restype = ctypes.c_uint32
        L.oracle_combine.argtypes = [ctypes.c_uint32, ctypes.c_uint32, ctypes.c_uint64]
        L.oracle_table_copy.restype = None
        L.oracle_table_copy.argtypes = [ctypes.c_void_p]
        _o = L
    return _o


def ref():
    """The compiled reference header, or None if oracle/_ref was not built."""
    global _r
    if _r is None and os.path.exists(REF_SO):
        L = ctypes.CDLL(REF_SO)
        L.ref_crc32c.restype = ctypes.c_uint32
        L.ref_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_uint]
        L.ref_table_copy.restype = None
        L.ref_table_copy.argtypes = [ctypes.c_void_p]
        if hasattr(L, "ref_crc32c_batch_mt"):
            L.ref_crc32c_batch_mt.restype = ctypes.c_int
            L.ref_crc32c_batch_mt.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p,
                                              ctypes.c_uint, ctypes.c_uint, ctypes.c_uint]
        L.ref_crc32c_strided.restype = None
        L.ref_crc32c_strided.argtypes = [ctypes.c_void_p, ctypes.c_ulong, ctypes.c_uint, ctypes.c_void_p,
                                         ctypes.c_uint]
        _r = L
    return _r


def crc(seed, data):
    a = np.frombuffer(bytes(data), dtype=np.uint8) if not isinstance(data, np.ndarray) else data
    a = np.ascontiguousarray(a)
    return oracle().oracle_crc32c(seed & 0xFFFFFFFF, a.ctypes.data, a.nbytes)


def crcs(host, offs, lens, seeds=None):
    """oracle CRC of host[off:off+len] for every (off, len): uint32 array."""
    host = np.ascontiguousarray(host, dtype=np.uint8)
    offs = np.asarray(offs, dtype=np.uint64)
    lens_u = np.ascontiguousarray(lens, dtype=np.uint32)
    n = len(lens_u)
    ptrs = (np.uint64(host.ctypes.data) + offs).astype(np.uint64)
    sd = None if seeds is None else np.ascontiguousarray(np.asarray(seeds, dtype=np.uint64) & 0xFFFFFFFF,
                                                          dtype=np.uint32)
    out = np.zeros(n, dtype=np.uint32)
    oracle().oracle_crc32c_batch(ptrs.ctypes.data, lens_u.ctypes.data, None if sd is None else sd.ctypes.data,
                                 out.ctypes.data, n)
    return out
