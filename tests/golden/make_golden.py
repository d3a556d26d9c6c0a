#!/usr/bin/env python3
"""Generate tests/golden/kat.json from the REFERENCE itself.

Run in the build container (needs /root/reference): it loads
oracle/_ref/libref_crc32c.so, which oracle/Makefile compiles from
/root/reference/include/crc32c.h (the reference's own crc32c(), :88-96), and
records inputs + expected outputs.  Inputs are described by a deterministic
generator (below) so the fixture stays small; the same generator lives in
tests/golden/gen.py for the tests to rebuild the bytes.

    make -C oracle ref && python tests/golden/make_golden.py
"""
import ctypes
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from gen import xorshift_bytes, splitmix_bytes  # noqa: E402

REPO = os.path.dirname(os.path.dirname(HERE))
LIB = os.path.join(REPO, "oracle", "_ref", "libref_crc32c.so")


def main():
    ref = ctypes.CDLL(LIB)
    ref.ref_crc32c.restype = ctypes.c_uint32
    ref.ref_crc32c.argtypes = [ctypes.c_uint32, ctypes.c_char_p, ctypes.c_uint]

    def crc(seed, data):
        return ref.ref_crc32c(seed, data, len(data))

    tab = (ctypes.c_uint32 * 256)()
    ref.ref_table_copy(tab)

    out = {
        "source": "oracle/_ref/libref_crc32c.so built from /root/reference/include/crc32c.h:88-96",
        "table": [int(x) for x in tab],
        "appendix_a": [],
        "vectors": [],
        "checks": {},
    }

    # xorshift32 data, fresh generator per row
    lens = [0, 1, 3, 4, 7, 8, 15, 16, 63, 64, 4095, 4096, 65536, 1048576, 4194304]
    seeds = [0x00000000, 0xFFFFFFFF, 0x12345678]
    for n in lens:
        d = xorshift_bytes(n)
        out["appendix_a"].append({"len": n, "crc": {f"{s:08x}": crc(s, d) for s in seeds}})

    # offset/length/seed sweep over a splitmix stream: covers unaligned starts,
    # ragged ends, tiny buffers and sizes straddling the 16/128/4096 B units
    # the GPU kernel is built around.
    stream = splitmix_bytes(0xC0FFEE, 3 * 65536 + 4096)
    cases = []
    for off in range(0, 33):
        for n in (0, 1, 2, 3, 4, 5, 13, 15, 16, 17, 31, 127, 128, 129, 255, 1000, 4095, 4096, 4097):
            cases.append((off, n))
    for off in (0, 1, 7, 15, 64, 100, 4095):
        for n in (8191, 8192, 16384 + 5, 65536, 65536 + 129, 131071):
            cases.append((off, n))
    for i, (off, n) in enumerate(cases):
        seed = [0, 0xFFFFFFFF, (0x9E3779B9 * (i + 1)) & 0xFFFFFFFF][i % 3]
        out["vectors"].append({"stream": "splitmix:0xC0FFEE", "off": off, "len": n,
                               "seed": seed, "crc": crc(seed, stream[off:off + n])})

    out["checks"] = {
        "123456789_seed0": crc(0, b"123456789"),
        "123456789_std": (~crc(0xFFFFFFFF, b"123456789")) & 0xFFFFFFFF,
        "zeros4096_seed0": crc(0, bytes(4096)),
        "ff4096_seed0": crc(0, b"\xff" * 4096),
        "zeros4096_seedffffffff": crc(0xFFFFFFFF, bytes(4096)),
    }
    path = os.path.join(HERE, "kat.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    print(f"wrote {path}: {len(out['appendix_a'])} appendix rows, {len(out['vectors'])} vectors")


if __name__ == "__main__":
    main()
