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

* the messenger adapter patch (integration/pech_crc32c_msgr.patch, the code
  of INTEGRATION.md §3.1-3.2) applies to temp copies of messenger.c,
  messenger.h and osd_server.c, compiles under the same flags, and the
  patched pech-osd links with every crc32c_* / crc32c_msgr_* symbol bound to
  the library.

Nothing is written under /root/reference and no object is kept."""
import glob
import os
import shutil
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


PATCH = os.path.join(REPO, "integration", "pech_crc32c_msgr.patch")
PATCHED = ("src/ceph/messenger.c", "include/ceph/messenger.h", "src/ceph/osd_server.c")


def compile_one(src, obj, with_dropin=True, extra_inc=()):
    inc = ((["-I" + os.path.join(REPO, "include")] if with_dropin else []) + ["-I" + d for d in extra_inc] +
           ["-I" + os.path.join(REF, "include")])
    return subprocess.run(["gcc", "-c", *CFLAGS, *inc, src, "-o", obj], capture_output=True, text=True, timeout=300)


def patched_tree(d):
    """Temp copies of the files the patch touches, patched; returns their root."""
    root = os.path.join(d, "pech")
    for rel in PATCHED:
        os.makedirs(os.path.dirname(os.path.join(root, rel)), exist_ok=True)
        shutil.copy(os.path.join(REF, rel), os.path.join(root, rel))
    r = subprocess.run(["patch", "-p1", "--no-backup-if-mismatch", "-d", root, "-i", PATCH], capture_output=True,
                       text=True, timeout=60)
    assert r.returncode == 0, r.stdout + r.stderr
    assert "fuzz" not in r.stdout and "offset" not in r.stdout, r.stdout  # applies exactly
    return root


def build_pech_osd(d, root=None):
    """Every src/**/*.c of pech compiled one by one into d (the patched copies
    from `root` in place of the originals), linked against the library."""
    srcs = sorted(glob.glob(os.path.join(REF, "src", "**", "*.c"), recursive=True))
    assert len(srcs) > 30
    if root:
        srcs = [os.path.join(root, os.path.relpath(s, REF)) if os.path.relpath(s, REF) in PATCHED else s
                for s in srcs]
    extra = [os.path.join(root, "include")] if root else []
    objs = [os.path.join(d, os.path.basename(os.path.dirname(s)) + "_" + os.path.basename(s)[:-2] + ".o")
            for s in srcs]
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        res = list(ex.map(lambda so: compile_one(*so, extra_inc=extra), zip(srcs, objs)))
    bad = [(s, r.stderr[-800:]) for s, r in zip(srcs, res) if r.returncode]
    assert not bad, bad[:2]
    exe = os.path.join(d, "pech-osd")
    r = subprocess.run(["gcc", "-o", exe, *objs, "-L" + LIBDIR, "-lpech_crc32c", "-Wl,-rpath," + LIBDIR,
                        "-lresolv", "-ldl", "-rdynamic"], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    return exe


def bindings(exe):
    """Run exe with every symbol bound at start-up; the dynamic linker's
    binding lines.  Without a monitor address pech-osd stops at option
    checking (main.c:253), before any GPU work."""
    env = dict(os.environ, LD_BIND_NOW="1", LD_DEBUG="bindings")
    r = subprocess.run([exe], capture_output=True, text=True, timeout=60, env=env)
    assert "mon_addrs" in r.stdout + r.stderr
    return r.stderr.splitlines()


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
    with tempfile.TemporaryDirectory() as d:
        lines = [l for l in bindings(build_pech_osd(d)) if "`crc32c'" in l]
        assert lines and all("libpech_crc32c.so" in l for l in lines), lines


# the library entry points the patched messenger calls
ADAPTER_SYMS = {"crc32c", "crc32c_async_create", "crc32c_async_fd", "crc32c_async_flush", "crc32c_async_complete",
                "crc32c_async_pending", "crc32c_async_destroy", "crc32c_last_error", "crc32c_msgr_conn_create",
                "crc32c_msgr_conn_destroy", "crc32c_msgr_conn_reset", "crc32c_msgr_rx_queue", "crc32c_msgr_rx_next",
                "crc32c_msgr_rx_pending", "crc32c_msgr_tx_submit", "crc32c_msgr_tx_has", "crc32c_msgr_tx_footer",
                "crc32c_msgr_tx_cancel", "crc32c_pages_alloc", "crc32c_pages_free", "crc32c_pages_is_pinned"}


def test_adapter_patch_compiles_against_the_reference():
    # the messenger patch on the adapter, against the real
    # struct ceph_connection and the real read/write/fault/revoke paths
    with tempfile.TemporaryDirectory() as d:
        root = patched_tree(d)
        for rel in ("src/ceph/messenger.c", "src/ceph/osd_server.c"):
            obj = os.path.join(d, os.path.basename(rel) + ".o")
            r = compile_one(os.path.join(root, rel), obj, extra_inc=[os.path.join(root, "include")])
            assert r.returncode == 0, (rel, r.stderr[-3000:])
            if rel.endswith("messenger.c"):
                und = {n for t, n in symbols(obj) if t == "U"}
                assert ADAPTER_SYMS <= und, ADAPTER_SYMS - und


def test_patched_pech_osd_binds_adapter_to_library():
    with tempfile.TemporaryDirectory() as d:
        lines = bindings(build_pech_osd(d, patched_tree(d)))
        for sym in ADAPTER_SYMS:
            got = [l for l in lines if f"`{sym}'" in l]
            assert got and all("libpech_crc32c.so" in l for l in got), (sym, got)


def test_integration_doc_carries_the_tested_patch():
    # INTEGRATION.md §3.1 shows exactly the patch these tests apply
    doc = open(os.path.join(REPO, "INTEGRATION.md")).read()
    body = open(PATCH).read()
    start = doc.index("```diff\n") + len("```diff\n")
    assert doc[start:doc.index("```", start)] == body
