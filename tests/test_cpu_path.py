"""The drop-in crc32c()'s host side (pech_amd/csrc/crc32c_cpu.c): the routine
that serves the messenger's small calls (49-byte
headers, front/middle sections, <=4 KiB data pieces) and keeps crc32c()
total when the GPU fails (§8(b) "Errors").  It must equal the reference
include/crc32c.h:88-96 on every golden vector, in both its SSE4.2 and its
portable form.  CPU tests; the GPU-box variants are marked gpu."""
import ctypes
import json
import os
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O
from gen import splitmix_bytes, xorshift_bytes

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KAT = json.load(open(os.path.join(REPO, "tests", "golden", "kat.json")))


_TEST_LIB = None


def L():
    """build/lib_test.so: the release objects plus the test hooks
    (-DPECH_TEST_HOOKS); the release library exports none of them."""
    global _TEST_LIB
    if _TEST_LIB is not None:
        return _TEST_LIB
    path = os.path.join(REPO, "build", "lib_test.so")
    assert os.path.exists(path), "build/lib_test.so is built by `make`"
    lib = ctypes.CDLL(path)
    lib.crc32c_test_cpu.restype = ctypes.c_uint32
    lib.crc32c_test_cpu.argtypes = [ctypes.c_uint32, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_int]
    lib.crc32c_test_cpu_has_sse42.restype = ctypes.c_int
    lib.crc32c_test_stack_switch.restype = ctypes.c_int
    _TEST_LIB = lib
    return lib


def cpu(seed, data, variant):
    a = np.ascontiguousarray(np.frombuffer(bytes(data), dtype=np.uint8)) if not isinstance(data, np.ndarray) else data
    return L().crc32c_test_cpu(seed & 0xFFFFFFFF, a.ctypes.data, a.size, variant)


VARIANTS = [0, 1]  # 0: what crc32c() uses (SSE4.2 here), 1: portable slice-by-8


@pytest.mark.parametrize("variant", VARIANTS)
def test_cpu_routine_appendix_a(variant):
    for row in KAT["appendix_a"]:
        d = xorshift_bytes(row["len"])
        for s, want in row["crc"].items():
            assert cpu(int(s, 16), d, variant) == want, (row["len"], s, variant)


@pytest.mark.parametrize("variant", VARIANTS)
def test_cpu_routine_offset_length_seed_vectors(variant):
    stream = np.frombuffer(splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096), dtype=np.uint8)
    lib = L()
    for v in KAT["vectors"]:
        got = lib.crc32c_test_cpu(v["seed"], stream.ctypes.data + v["off"], v["len"], variant)
        assert got == v["crc"], (v, variant)


@pytest.mark.parametrize("variant", VARIANTS)
def test_cpu_routine_checks(variant):
    c = KAT["checks"]
    assert cpu(0, b"123456789", variant) == c["123456789_seed0"]
    assert cpu(0, bytes(4096), variant) == c["zeros4096_seed0"]
    assert cpu(0, b"\xff" * 4096, variant) == c["ff4096_seed0"]
    assert cpu(0xFFFFFFFF, bytes(4096), variant) == c["zeros4096_seedffffffff"]


def test_cpu_routine_block_edges():
    # the 3-stream rounds (3 x 8 KiB, then 3 x 256 B) and the 8-byte tail,
    # at every alignment of the start
    rng = np.random.default_rng(21)
    big = rng.integers(0, 256, 3 * 8192 * 3 + 64, dtype=np.uint8)
    for n in (0, 1, 7, 8, 9, 767, 768, 769, 24575, 24576, 24577, 24576 + 768, 49152 + 5, 3 * 8192 * 3):
        for off in range(0, 9):
            s = int(rng.integers(0, 1 << 32))
            d = big[off:off + n]
            want = O.crc(s, d)
            assert cpu(s, d, 0) == want, (n, off)
            assert cpu(s, d, 1) == want, (n, off)


def test_dropin_is_total_without_gpu():
    # No GPU in this container: calls up to the CPU threshold never touch
    # HIP; a larger call fails its GPU leg and is recomputed on the host.
    # Replaces r01's "abort without a GPU".  Subprocess: no HIP state here.
    code = r"""
import ctypes, sys, json
import numpy as np
sys.path.insert(0, "tests")
import oracle_lib as O
from pech_amd import _lib
L = _lib.lib()
rng = np.random.default_rng(4)
res = []
for n in (1, 49, 4096, 65536, 1 << 20):
    d = rng.integers(0, 256, n, dtype=np.uint8)
    s = int(rng.integers(0, 1 << 32))
    res.append(L.crc32c(s, d.ctypes.data, n) == O.crc(s, d))
L.crc32c_set_cpu_max.restype = ctypes.c_uint
L.crc32c_set_cpu_max.argtypes = [ctypes.c_uint]
prev = L.crc32c_set_cpu_max(1000)
d = rng.integers(0, 256, 5000, dtype=np.uint8)
res.append(L.crc32c(7, d.ctypes.data, 5000) == O.crc(7, d))   # GPU leg fails -> host
from pech_amd import stats
print(json.dumps({"ok": res, "prev": prev, "stats": stats()}))
"""
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, timeout=300)
    if os.path.exists("/dev/kfd"):
        pytest.skip("a GPU is present: the fallback leg would not fail")
    assert r.returncode == 0, r.stderr.decode()
    out = json.loads(r.stdout.decode().strip().splitlines()[-1])
    assert all(out["ok"]), out
    assert out["prev"] == 4 << 20
    st = out["stats"]
    assert st["gpu_calls"] == 0 and st["gpu_fallbacks"] == 1 and st["cpu_calls"] == 6, st
    assert b"computing on the CPU" in r.stderr


def test_cpu_max_from_environment():
    code = ("import ctypes\nfrom pech_amd import _lib\nL=_lib.lib()\n"
            "L.crc32c_set_cpu_max.restype=ctypes.c_uint\nprint(L.crc32c_set_cpu_max(5))\n")
    env = dict(os.environ, PECH_CRC32C_CPU_MAX="12345")
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, timeout=120, env=env)
    assert r.returncode == 0, r.stderr.decode()
    assert int(r.stdout.decode().split()[-1]) == 12345


def test_library_stack_switch():
    # every HIP-calling entry point runs on the per-thread library stack
    assert L().crc32c_test_stack_switch() == 1


def test_no_oracle_in_product():
    # the product library neither links nor contains the test oracle
    from pech_amd import _lib

    syms = subprocess.check_output(["nm", "-D", _lib.LIB_PATH]).decode()
    assert "oracle_" not in syms
    syms_all = subprocess.check_output(["nm", _lib.LIB_PATH]).decode()
    assert "oracle_" not in syms_all
    deps = subprocess.check_output(["readelf", "-d", _lib.LIB_PATH]).decode()
    assert "oracle" not in deps


@pytest.mark.gpu
def test_cpu_routine_every_vector_on_gpu_host():
    # the same checks on the GPU box's own CPU (the routine the drop-in uses there)
    for variant in VARIANTS:
        test_cpu_routine_appendix_a(variant)
        test_cpu_routine_offset_length_seed_vectors(variant)
        test_cpu_routine_checks(variant)
    test_cpu_routine_block_edges()


@pytest.mark.gpu
def test_coroutine_stack_64k():
    # gnu89 C: crc32c() (host and GPU routes), crc32c_batch and the async
    # layer called from a task on a 64 KiB stack with a guard page, as pech's
    # workqueue runs the messenger (src/sched.c:16, :120-128)
    exe = os.path.join(REPO, "build", "coro_stack")
    assert os.path.exists(exe), "build/coro_stack is built by `make`"
    r = subprocess.run([exe, "64"], capture_output=True, timeout=300)
    out = r.stdout.decode()
    assert r.returncode == 0, (out, r.stderr.decode())
    hwm = int(out.split("hwm")[1].split()[0])
    print("coroutine stack high-water mark with the library stack:", hwm)
    assert hwm < 32 << 10
    # what the same calls need WITHOUT the library stack (diagnostic, on a
    # 4 MiB task stack so that it cannot overflow)
    env = dict(os.environ, PECH_STACK_SWITCH="0")
    r2 = subprocess.run([exe, "4096"], capture_output=True, timeout=300, env=env)
    assert r2.returncode == 0, (r2.stdout, r2.stderr)
    print("without the library stack:", r2.stdout.decode().strip())
