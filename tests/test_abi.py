"""The C-ABI library: loads, exports every function include/*.h declares, and
its host-side algebra (shift/combine, no data pass) matches the oracle.
No GPU compute calls here -- those need a GPU (tests/test_gpu_parity.py)."""
import ctypes
import os
import re
import subprocess
import sys

import numpy as np
import pytest

import oracle_lib as O

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
INCLUDE = os.path.join(REPO, "include")


def declared_functions():
    names = set()
    for h in os.listdir(INCLUDE):
        if not h.endswith(".h"):
            continue
        src = open(os.path.join(INCLUDE, h)).read()
        src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
        for m in re.finditer(r"^[A-Za-z_][\w \*]*?\b(crc32c\w*)\s*\(", src, flags=re.M):
            names.add(m.group(1))
    return names


def test_header_declares_dropin():
    names = declared_functions()
    assert "crc32c" in names
    assert {"crc32c_batch", "crc32c_dev_batch_async", "crc32c_combine", "crc32c_shift"} <= names


def test_library_exports_every_declared_symbol():
    from pech_amd import _lib

    L = _lib.lib()
    for name in declared_functions():
        assert hasattr(L, name), name
    assert set(_lib.SIGNATURES) >= declared_functions()
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    exported = {line.split()[-1] for line in out.splitlines() if " T " in line}
    assert declared_functions() <= exported


def test_dropin_header_compiles_as_pech_c():
    # pech is gnu89 C (reference Makefile); the drop-in must compile there
    src = '#include "crc32c.h"\n#include "pech_crc32c.h"\nint main(void){return (int)sizeof(struct crc32c_desc)-16;}\n'
    exe = os.path.join(REPO, "build", "hdrcheck")
    os.makedirs(os.path.dirname(exe), exist_ok=True)
    r = subprocess.run(["gcc", "-std=gnu89", "-Wall", "-Werror", "-I" + INCLUDE, "-x", "c", "-", "-o", exe],
                       input=src.encode(), capture_output=True)
    assert r.returncode == 0, r.stderr.decode()
    assert subprocess.run([exe]).returncode == 0


def test_shift_combine_match_oracle():
    from pech_amd import crc32c_combine, crc32c_shift

    o = O.oracle()
    rng = np.random.default_rng(5)
    for _ in range(200):
        v = int(rng.integers(0, 1 << 32))
        n = int(rng.integers(0, 1 << 40))
        assert crc32c_shift(v, n) == o.oracle_shift(v, n)
        b = int(rng.integers(0, 1 << 32))
        assert crc32c_combine(v, b, n) == o.oracle_combine(v, b, n)
    a = rng.integers(0, 256, 5000, dtype=np.uint8)
    assert crc32c_combine(O.crc(9, a[:1234]), O.crc(0, a[1234:]), 5000 - 1234) == O.crc(9, a)


def test_batch_flag_validation():
    # checked before any device work: runs with or without a GPU
    from pech_amd import _lib

    L = _lib.lib()
    buf = ctypes.create_string_buffer(b"abc")
    p = (ctypes.c_void_p * 1)(ctypes.addressof(buf))
    l = (ctypes.c_uint * 1)(3)
    out = (ctypes.c_uint32 * 1)()
    for flags in (3, 4, 5, 7, 8, 1 | 4):  # DEVICE|PINNED, ALL_DEVICES without PINNED, unknown bits
        assert L.crc32c_batch(p, l, None, out, 1, flags) == -22, flags


@pytest.mark.skipif(os.path.exists("/dev/kfd"), reason="checks the no-GPU failure mode")
def test_no_gpu_batch_fails_loudly():
    # without a GPU the batch API returns an error: the throughput path has no
    # CPU fallback.  (The drop-in crc32c() stays total instead, like the
    # reference: tests/test_cpu_path.py::test_dropin_is_total_without_gpu.)
    code = (
        "import ctypes, sys\n"
        "from pech_amd import _lib\n"
        "L = _lib.lib()\n"
        "out = (ctypes.c_uint32 * 1)()\n"
        "p = (ctypes.c_void_p * 1)(ctypes.addressof(ctypes.create_string_buffer(b'abc')))\n"
        "l = (ctypes.c_uint * 1)(3)\n"
        "rc = L.crc32c_batch(p, l, None, out, 1, 0)\n"
        "print(rc, L.crc32c_last_error().decode())\n"
        "sys.exit(0 if rc < 0 else 1)\n"
    )
    r = subprocess.run([sys.executable, "-c", code], cwd=REPO, capture_output=True, timeout=120)
    assert r.returncode == 0, (r.stdout, r.stderr)


def _xorshift_bytes(n):
    # SURVEY Appendix A's generator (tests/c/dropin_kat.c gen())
    out = np.empty(n, np.uint8)
    s = 0x2545F491
    for i in range(n):
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        out[i] = s & 0xFF
    return out


def test_dropin_kat_builds_as_pech_c():
    r = subprocess.run(["make", "-s", "-C", REPO, "build/dropin_kat"], capture_output=True)
    assert r.returncode == 0, r.stderr.decode()


@pytest.mark.gpu
@pytest.mark.parametrize("cpu_max", [None, "0"])
def test_dropin_from_c_matches_appendix_a(cpu_max):
    # the drop-in called from gnu89 C (one call, the <=4 KiB page-piece chain
    # of ceph_crc32c_iov, a 49-byte header call) against the golden vectors
    # the compiled reference produced (tests/golden/kat.json)
    import json

    kat = json.load(open(os.path.join(REPO, "tests", "golden", "kat.json")))
    exe = os.path.join(REPO, "build", "dropin_kat")
    assert os.path.exists(exe), "build/dropin_kat is built by `make` (__graft_entry__.build())"
    args, want = [], {}
    for e in kat["appendix_a"]:
        for seed_hex, crc in e["crc"].items():
            args.append("%d:%s" % (e["len"], seed_hex))
            want[(e["len"], int(seed_hex, 16))] = crc
    # cpu_max None: the default routing (host routine up to 4 MiB, GPU above);
    # "0": every non-empty call through the gfx950 kernels
    env = dict(os.environ)
    if cpu_max is not None:
        env["PECH_CRC32C_CPU_MAX"] = cpu_max
    r = subprocess.run([exe] + args, capture_output=True, timeout=300, env=env)
    assert r.returncode == 0, (r.stdout, r.stderr)
    fields = r.stdout.decode().split()
    rows = [fields[i:i + 5] for i in range(0, len(fields), 5)]
    assert len(rows) == len(args)
    hdr_want = {}
    for n, seed, whole, pieces, hdr in rows:
        n, seed = int(n), int(seed, 16)
        assert int(whole, 16) == want[(n, seed)], (n, seed)
        assert int(pieces, 16) == want[(n, seed)], (n, seed)
        if n not in hdr_want:
            hdr_want[n] = O.crc(0, _xorshift_bytes(min(n, 49)))
        assert int(hdr, 16) == hdr_want[n], n
