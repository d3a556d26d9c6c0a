"""Deterministic input generators shared by the golden-vector script, the
tests and bench.py (which fills device buffers with the same splitmix words
on the GPU, so any buffer can be rebuilt on the host for a spot check)."""
import numpy as np

M64 = (1 << 64) - 1
GAMMA = 0x9E3779B97F4A7C15
STEP = 0xD1B54A32D192ED03


def xorshift_bytes(n, state=0x2545F491):
    """SURVEY.md Appendix A generator: xorshift32, one byte per update."""
    out = bytearray(n)
    s = state
    for i in range(n):
        s ^= (s << 13) & 0xFFFFFFFF
        s ^= s >> 17
        s ^= (s << 5) & 0xFFFFFFFF
        out[i] = s & 0xFF
    return bytes(out)


def fmix64(z):
    """splitmix64 finalizer on a uint64 numpy array (wrapping arithmetic)."""
    z = z.astype(np.uint64)
    with np.errstate(over="ignore"):
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        z = z ^ (z >> np.uint64(31))
    return z


def splitmix_words(key, nwords, first=0):
    """word j = fmix64(key*GAMMA + (j+1)*STEP), j in [first, first+nwords)."""
    j = np.arange(first, first + nwords, dtype=np.uint64)
    with np.errstate(over="ignore"):
        x = np.uint64((key * GAMMA) & M64) + (j + np.uint64(1)) * np.uint64(STEP)
    return fmix64(x)


def splitmix_bytes(key, n):
    w = splitmix_words(key, (n + 7) // 8)
    return w.astype("<u8").tobytes()[:n]
