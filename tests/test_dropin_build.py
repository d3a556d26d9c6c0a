"""The drop-in claim, checked against the reference's own sources (build
container only: /root/reference does not exist on the GPU box).

* src/ceph/messenger.c -- the only caller of crc32c() (include at :6, six
  call sites) -- compiles UNCHANGED with this repo's include/ ahead of the
  reference's, with the reference Makefile's CFLAGS (-std=gnu89 -Werror ...),
  and then references an external `crc32c` (the reference's is static
  inline, so its object has none);
* all of pech (every src/**/*.c, compiled one by one into a temp dir -- not
  the reference's build system) links into pech-osd against
  libpech_crc32c.so, and the dynamic linker binds the messenger's crc32c to
  the library.

Nothing is written under /root/reference and no object is kept."""
import glob
import os
import subprocess
import tempfile
from concurrent.futures import ThreadPoolExecutor

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
LIBDIR = os.path.join(REPO, "pech_amd")

pytestmark = pytest.mark.skipif(not os.path.isdir(os.path.join(REF, "src", "ceph")),
                                reason="needs the reference sources (build container only)")

# the reference Makefile's CFLAGS (Makefile:2-12); gcc 11 also needs
# unused-result demoted (include/random.h:10) and _FORTIFY_SOURCE off for
# pech's cross-stack longjmp
CFLAGS = ["-g", "-O2", "-std=gnu89", "-Wall", "-Wdeclaration-after-statement", "-Wno-format", "-Werror",
          "-Werror=date-time", "-Werror=incompatible-pointer-types", "-Werror=designated-init",
          "-Wno-unused-const-variable", "-Wno-unused-but-set-variable", "-Wno-pointer-sign", "-fno-strict-aliasing",
          "-fstack-protector-strong", "-Wno-error=unused-result", "-U_FORTIFY_SOURCE", "-D_FORTIFY_SOURCE=0",
          "-D_GNU_SOURCE", "-D__KERNEL__"]


def compile_one(src, obj, with_dropin=True):
    inc = (["-I" + os.path.join(REPO, "include")] if with_dropin else []) + ["-I" + os.path.join(REF, "include")]
    return subprocess.run(["gcc", "-c", *CFLAGS, *inc, src, "-o", obj], capture_output=True, text=True, timeout=300)


def symbols(obj):
    out = subprocess.check_output(["nm", obj]).decode()
    return {(l.split()[-2], l.split()[-1]) for l in out.splitlines() if len(l.split()) >= 2}


def test_messenger_compiles_unchanged():
    src = os.path.join(REF, "src", "ceph", "messenger.c")
    with tempfile.TemporaryDirectory() as d:
        obj = os.path.join(d, "messenger.o")
        r = compile_one(src, obj)
        assert r.returncode == 0, r.stderr[-3000:]
        syms = symbols(obj)
        assert ("U", "crc32c") in syms              # calls the library's exported symbol
        assert not any(n == "crc32c" and t in "Tt" for t, n in syms)
        # control: with the reference header the function is inlined
        ref_obj = os.path.join(d, "messenger_ref.o")
        r = compile_one(src, ref_obj, with_dropin=False)
        assert r.returncode == 0, r.stderr[-3000:]
        assert ("U", "crc32c") not in symbols(ref_obj)
    lib = os.path.join(LIBDIR, "libpech_crc32c.so")
    out = subprocess.check_output(["nm", "-D", "--defined-only", lib]).decode()
    assert any(l.split()[-1] == "crc32c" and l.split()[-2] == "T" for l in out.splitlines())


def test_pech_osd_links_and_binds_to_library():
    srcs = sorted(glob.glob(os.path.join(REF, "src", "**", "*.c"), recursive=True))
    assert len(srcs) > 30
    with tempfile.TemporaryDirectory() as d:
        objs = [os.path.join(d, os.path.relpath(s, os.path.join(REF, "src")).replace("/", "_")[:-2] + ".o")
                for s in srcs]
        with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
            res = list(ex.map(lambda so: compile_one(*so), zip(srcs, objs)))
        bad = [(s, r.stderr[-800:]) for s, r in zip(srcs, res) if r.returncode]
        assert not bad, bad[:2]
        exe = os.path.join(d, "pech-osd")
        r = subprocess.run(["gcc", "-o", exe, *objs, "-L" + LIBDIR, "-lpech_crc32c", "-Wl,-rpath," + LIBDIR,
                            "-lresolv", "-ldl", "-rdynamic"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr[-3000:]
        # bind every symbol at start-up and ask the dynamic linker where crc32c went;
        # without a monitor address pech-osd stops at option checking (main.c:253)
        env = dict(os.environ, LD_BIND_NOW="1", LD_DEBUG="bindings")
        r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=env)
        lines = [l for l in r.stderr.splitlines() if "`crc32c'" in l]
        assert lines and all("libpech_crc32c.so" in l for l in lines), lines or r.stderr[-2000:]
        assert "mon_addrs" in r.stdout + r.stderr
