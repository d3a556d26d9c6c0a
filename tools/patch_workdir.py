"""Edit the messenger patch as code (build container only).

    python3 tools/patch_workdir.py export /tmp/pw   # /tmp/pw/a (reference), /tmp/pw/b (patched)
    ... edit /tmp/pw/b/src/ceph/messenger.c etc ...
    python3 tools/patch_workdir.py diff /tmp/pw     # -> integration/pech_crc32c_msgr.patch, INTEGRATION.md §3.1

The work directory must lie outside the repository: it holds copies of
reference sources, which never enter this tree.
"""
import os
import shutil
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tests"))
import pech_build as B  # noqa: E402


def export(d):
    if os.path.abspath(d).startswith(REPO + os.sep):
        sys.exit("the work directory must be outside the repository")
    os.makedirs(d, exist_ok=True)
    for side in ("a", "b"):
        shutil.rmtree(os.path.join(d, side), ignore_errors=True)
    for rel in B.PATCHED:
        dst = os.path.join(d, "a", rel)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        shutil.copy(os.path.join(B.REF, rel), dst)
    root = B.patched_tree(d)
    os.rename(root, os.path.join(d, "b"))


def diff(d):
    out = []
    for rel in sorted(B.PATCHED, key=lambda r: (not r.endswith(".h"), r)):  # the header first
        r = subprocess.run(["diff", "-u", "--label", "a/" + rel, "--label", "b/" + rel, os.path.join(d, "a", rel),
                            os.path.join(d, "b", rel)], capture_output=True, text=True)
        if r.returncode not in (0, 1):
            sys.exit(r.stderr)
        out.append(r.stdout)
    open(B.PATCH, "w").write("".join(out))
    subprocess.check_call([sys.executable, os.path.join(REPO, "tools", "sync_integration.py")])


if __name__ == "__main__":
    if len(sys.argv) != 3 or sys.argv[1] not in ("export", "diff"):
        sys.exit(__doc__)
    {"export": export, "diff": diff}[sys.argv[1]](sys.argv[2])
