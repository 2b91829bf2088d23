"""Portable counter-based PRNG (splitmix64) used to build deterministic weights.

The same hash is implemented on the device (`mtts_fill_uniform_bf16` in
`moss_tts_amd/csrc/init_kernels.hip`), so a weight tensor is fully described
by (seed, tensor_id, scale, offset) and the golden fixtures need to carry
only seeds and outputs, never weights.

    z   = splitmix64(seed * GOLDEN + (tensor_id << 40) + i)
    u   = (z >> 40) * 2^-24            # uniform in [0, 1)
    val = offset + scale * (2u - 1)
"""
import numpy as np

_GOLDEN = np.uint64(0x9E3779B97F4A7C15)
_M1 = np.uint64(0xBF58476D1CE4E5B9)
_M2 = np.uint64(0x94D049BB133111EB)


def splitmix64(x):
    x = np.asarray(x, dtype=np.uint64)
    with np.errstate(over="ignore"):
        z = x + _GOLDEN
        z = (z ^ (z >> np.uint64(30))) * _M1
        z = (z ^ (z >> np.uint64(27))) * _M2
        z = z ^ (z >> np.uint64(31))
    return z


def uniform(seed, tensor_id, n, start=0):
    """n uniforms in [0,1) as float32 for counters start..start+n-1."""
    with np.errstate(over="ignore"):
        base = np.uint64(seed) * _GOLDEN + (np.uint64(tensor_id) << np.uint64(40))
        ctr = base + np.arange(start, start + n, dtype=np.uint64)
    z = splitmix64(ctr)
    return ((z >> np.uint64(40)).astype(np.float32) * np.float32(2.0 ** -24)).astype(np.float32)


def tensor(seed, tensor_id, shape, scale, offset=0.0):
    n = int(np.prod(shape))
    u = uniform(seed, tensor_id, n)
    v = np.float32(offset) + np.float32(scale) * (np.float32(2.0) * u - np.float32(1.0))
    return v.astype(np.float32).reshape(shape)


_M32 = 0xFFFFFFFF


def philox_uniform(seed, c0, c1, c2):
    """Philox4x32-10 uniform in [0, 1) with 24 bits: the counter-based draw the samplers use
    (`moss_tts_amd/csrc/common.h` philox_uniform; counters (step, row, channel), key = seed).
    Pure-Python integers (test infrastructure only)."""
    x0, x1, x2, x3 = int(c0) & _M32, int(c1) & _M32, int(c2) & _M32, 0x5EED
    k0, k1 = int(seed) & _M32, (int(seed) >> 32) & _M32
    for _ in range(10):
        p0 = 0xD2511F53 * x0
        p1 = 0xCD9E8D57 * x2
        h0, l0 = p0 >> 32, p0 & _M32
        h1, l1 = p1 >> 32, p1 & _M32
        x0, x1, x2, x3 = h1 ^ x1 ^ k0, l1, h0 ^ x3 ^ k1, l0
        k0 = (k0 + 0x9E3779B9) & _M32
        k1 = (k1 + 0xBB67AE85) & _M32
    return np.float32(x0 >> 8) * np.float32(1.0 / 16777216.0)
