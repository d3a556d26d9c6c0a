"""Compile pech's own sources (/root/reference, read-only) against this repo's
include/ -- unchanged or patched by integration/pech_crc32c_msgr.patch -- in
a temporary directory, with the reference Makefile's CFLAGS (Makefile:2-12),
one file at a time (not the reference's build system).  Used by
tests/test_dropin_build.py and, through `make build/msgr_loopback`, to link
tests/c/msgr_loopback.c against the patched messenger.

Only in the build container: /root/reference does not exist on the GPU box.
Patched copies and objects live in a temp dir that is removed afterwards;
the only output kept is the linked test binary (build/msgr_loopback), which
travels to the GPU box like oracle/_ref.

    python3 tests/pech_build.py loopback build/msgr_loopback
"""
import glob
import os
import shutil
import subprocess
import sys
import tempfile
from concurrent.futures import ThreadPoolExecutor

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF = "/root/reference"
LIBDIR = os.path.join(REPO, "pech_amd")
PATCH = os.path.join(REPO, "integration", "pech_crc32c_msgr.patch")
PATCHED = ("src/ceph/messenger.c", "include/ceph/messenger.h", "src/ceph/osd_server.c")

# the reference Makefile's CFLAGS (Makefile:2-12); gcc 11 also needs
# unused-result demoted (include/random.h:10) and _FORTIFY_SOURCE off for
# pech's cross-stack longjmp
CFLAGS = ["-g", "-O2", "-std=gnu89", "-Wall", "-Wdeclaration-after-statement", "-Wno-format", "-Werror",
          "-Werror=date-time", "-Werror=incompatible-pointer-types", "-Werror=designated-init",
          "-Wno-unused-const-variable", "-Wno-unused-but-set-variable", "-Wno-pointer-sign", "-fno-strict-aliasing",
          "-fstack-protector-strong", "-Wno-error=unused-result", "-U_FORTIFY_SOURCE", "-D_FORTIFY_SOURCE=0",
          "-D_GNU_SOURCE", "-D__KERNEL__"]


def have_reference():
    return os.path.isdir(os.path.join(REF, "src", "ceph"))


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
    if r.returncode != 0:
        raise RuntimeError("patch failed: " + r.stdout + r.stderr)
    if "fuzz" in r.stdout or "offset" in r.stdout:
        raise RuntimeError("patch does not apply exactly: " + r.stdout)
    return root


def pech_objects(d, root=None, skip_main=False):
    """Every src/**/*.c of pech compiled one by one into d (the patched copies
    from `root` in place of the originals); returns the object paths."""
    srcs = sorted(glob.glob(os.path.join(REF, "src", "**", "*.c"), recursive=True))
    if len(srcs) <= 30:
        raise RuntimeError("pech sources not found")
    if skip_main:
        srcs = [s for s in srcs if os.path.relpath(s, REF) != "src/main.c"]
    if root:
        srcs = [os.path.join(root, os.path.relpath(s, REF)) if os.path.relpath(s, REF) in PATCHED else s
                for s in srcs]
    extra = [os.path.join(root, "include")] if root else []
    objs = [os.path.join(d, os.path.basename(os.path.dirname(s)) + "_" + os.path.basename(s)[:-2] + ".o")
            for s in srcs]
    with ThreadPoolExecutor(max_workers=min(8, os.cpu_count() or 4)) as ex:
        res = list(ex.map(lambda so: compile_one(*so, extra_inc=extra), zip(srcs, objs)))
    bad = [(s, r.stderr[-800:]) for s, r in zip(srcs, res) if r.returncode]
    if bad:
        raise RuntimeError(f"pech source failed to compile: {bad[:2]}")
    return objs


LINK_LIBS = ["-L" + LIBDIR, "-lpech_crc32c", "-lresolv", "-ldl", "-lpthread", "-rdynamic"]


def build_pech_osd(d, root=None):
    """pech-osd itself, linked against the library (rpath to pech_amd/)."""
    objs = pech_objects(d, root)
    exe = os.path.join(d, "pech-osd")
    r = subprocess.run(["gcc", "-o", exe, *objs, *LINK_LIBS, "-Wl,-rpath," + LIBDIR], capture_output=True,
                       text=True, timeout=300)
    if r.returncode != 0:
        raise RuntimeError(r.stderr[-3000:])
    return exe


def build_loopback(out):
    """build/msgr_loopback: tests/c/msgr_loopback.c + the relay + the test
    oracle, linked with every pech object but main.c (patched messenger) and
    the library, with an rpath relative to the binary so it runs from the
    GPU box's copy of the tree."""
    with tempfile.TemporaryDirectory() as d:
        root = patched_tree(d)
        objs = pech_objects(d, root, skip_main=True)
        tc = os.path.join(REPO, "tests", "c")
        lb = os.path.join(d, "msgr_loopback.o")
        r = compile_one(os.path.join(tc, "msgr_loopback.c"), lb, extra_inc=[os.path.join(root, "include"), tc])
        if r.returncode:
            raise RuntimeError(r.stderr[-3000:])
        px = os.path.join(d, "loopback_proxy.o")
        orc = os.path.join(d, "crc32c_oracle.o")
        for src, obj, std in ((os.path.join(tc, "loopback_proxy.c"), px, "gnu11"),
                              (os.path.join(REPO, "oracle", "crc32c_oracle.c"), orc, "gnu11")):
            r = subprocess.run(["gcc", "-c", "-O2", "-std=" + std, "-Wall", "-Werror", src, "-o", obj],
                               capture_output=True, text=True, timeout=120)
            if r.returncode:
                raise RuntimeError(r.stderr[-3000:])
        os.makedirs(os.path.dirname(os.path.abspath(out)), exist_ok=True)
        tmp = out + ".tmp"
        # the test wraps the messenger's held-footer call, its socket
        # writes and its complete() calls (the revoke scenario holds the
        # target's send until it is revoked) and its context creation (the
        # contexts' counters)
        r = subprocess.run(["gcc", "-o", tmp, lb, px, orc, *objs, *LINK_LIBS, "-Wl,-rpath,$ORIGIN/../pech_amd",
                            "-Wl,--wrap=crc32c_msgr_tx_footer", "-Wl,--wrap=crc32c_async_create_on",
                            "-Wl,--wrap=sock_sendmsg", "-Wl,--wrap=crc32c_async_complete"],
                           capture_output=True, text=True, timeout=300)
        if r.returncode:
            raise RuntimeError(r.stderr[-3000:])
        os.replace(tmp, out)
    return out


if __name__ == "__main__":
    if len(sys.argv) != 3 or sys.argv[1] != "loopback":
        sys.exit(__doc__)
    if not have_reference():
        sys.exit("pech_build: /root/reference is not here (build container only)")
    print(build_loopback(sys.argv[2]))
