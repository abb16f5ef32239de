"""Deterministic synthetic inputs shared by tests and bench (SURVEY.md §8d definitions)."""
import numpy as np

M64 = (1 << 64) - 1


def splitmix64(x: np.ndarray) -> np.ndarray:
    x = (x + np.uint64(0x9E3779B97F4A7C15)) & np.uint64(M64)
    z = x
    z = ((z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)) & np.uint64(M64)
    z = ((z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)) & np.uint64(M64)
    return z ^ (z >> np.uint64(31))


def gen_f32(start: int, count: int) -> np.ndarray:
    """gen_f32: x = 20 + 5 sin(2pi (g mod 4096)/4096) + ((splitmix64(1234^g)>>40) 2^-24) 0.01,
    computed in float32 for global element index g."""
    g = np.arange(start, start + count, dtype=np.uint64)
    with np.errstate(over="ignore"):
        r = splitmix64(np.uint64(1234) ^ g)
    noise = (r >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24) * np.float32(0.01)
    ph = (g % np.uint64(4096)).astype(np.float32) * np.float32(2 * np.pi / 4096)
    return (np.float32(20) + np.float32(5) * np.sin(ph).astype(np.float32) + noise).astype(np.float32)


def int64_ramp(start: int, count: int) -> np.ndarray:
    """C4 input: value = global element index."""
    return np.arange(start, start + count, dtype=np.int64)


def b2bench_values(n: int, rshift: int = 19) -> np.ndarray:
    """bench/b2bench.c:73-81 get_value(i, rshift): (i<<26)^(i<<18)^(i<<11)^(i<<3)^i masked to rshift bits,
    computed in 32-bit int arithmetic."""
    i = np.arange(n, dtype=np.uint32)
    v = (i << np.uint32(26)) ^ (i << np.uint32(18)) ^ (i << np.uint32(11)) ^ (i << np.uint32(3)) ^ i
    if rshift < 32:
        v &= np.uint32((1 << rshift) - 1)
    return v.view(np.int32)


def mixed_bytes(seed: int, nbytes: int) -> np.ndarray:
    """Byte stream with runs, repeats and noise: exercises literals, near/far/long matches and runs."""
    rng = np.random.default_rng(seed)
    out = np.empty(nbytes, np.uint8)
    pos = 0
    while pos < nbytes:
        kind = rng.integers(0, 5)
        n = int(rng.integers(1, 600))
        n = min(n, nbytes - pos)
        if kind == 0:
            out[pos:pos + n] = rng.integers(0, 256, n, dtype=np.uint8)
        elif kind == 1:
            out[pos:pos + n] = rng.integers(0, 256, dtype=np.uint8)
        elif kind == 2 and pos > 0:
            d = int(rng.integers(1, min(pos, 80000) + 1))
            for k in range(n):
                out[pos + k] = out[pos + k - d]
        elif kind == 3:
            out[pos:pos + n] = 0
        else:
            out[pos:pos + n] = (np.arange(n) // int(rng.integers(1, 9))).astype(np.uint8)
        pos += n
    return out
