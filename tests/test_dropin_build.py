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
import os
import subprocess
import tempfile

import pytest

import pech_build as B
from pech_build import LIBDIR, PATCH, REF, REPO, build_pech_osd, compile_one, patched_tree

pytestmark = pytest.mark.skipif(not B.have_reference(), reason="needs the reference sources (build container only)")


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
ADAPTER_SYMS = {"crc32c", "crc32c_async_devices", "crc32c_async_create_on", "crc32c_msgr_conn_async", "crc32c_async_fd", "crc32c_async_flush", "crc32c_async_complete",
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
