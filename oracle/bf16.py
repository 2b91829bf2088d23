"""bf16 emulation on float32 numpy arrays (oracle / test infrastructure only).

The reference runs in bf16 with fp32 internals at specific points (SURVEY.md
fact 6).  `rnd` rounds float32 values to the nearest bf16 value (ties to
even), returning float32 arrays whose values are exactly bf16-representable,
which is what torch does on every bf16 op output.
"""
import numpy as np


def rnd(x):
    """Round float32 -> nearest bf16 (RNE), returned as float32. NaN stays NaN."""
    a = np.ascontiguousarray(np.asarray(x, dtype=np.float32))
    u = a.view(np.uint32).astype(np.uint64)
    lsb = (u >> np.uint64(16)) & np.uint64(1)
    r = ((u + np.uint64(0x7FFF) + lsb) >> np.uint64(16)) << np.uint64(16)
    out = r.astype(np.uint32).view(np.float32).reshape(a.shape)
    nan = np.isnan(a)
    if nan.any():
        out = out.copy()
        out[nan] = np.nan
    return out


def to_bits(x):
    """float32 (bf16-representable) -> uint16 bf16 bit pattern."""
    a = rnd(x)
    return (a.view(np.uint32) >> np.uint32(16)).astype(np.uint16)


def from_bits(b):
    """uint16 bf16 bits -> float32."""
    b = np.asarray(b, dtype=np.uint16)
    return (b.astype(np.uint32) << np.uint32(16)).view(np.float32)
