"""Helpers shared by the parity tests (trajectory comparison with a bf16 band)."""
import numpy as np

from oracle import bf16 as B16


def ulp_bf16(x):
    """bf16 ulp at |x| (float32 in, float32 out)."""
    a = np.abs(np.asarray(x, np.float32))
    a = np.where(a < 2.0 ** -126, 2.0 ** -126, a)
    e = np.floor(np.log2(a))
    return (2.0 ** (e - 7)).astype(np.float32)


def margin_top2(row):
    """top1 - top2 of a finite-max logit row (0 if ties)."""
    r = np.asarray(row, np.float64)
    r = r[np.isfinite(r)]
    if r.size < 2:
        return np.inf
    p = np.partition(r, -2)
    return float(p[-1] - p[-2])


def first_divergence(out_a, out_b):
    """index of the first differing row of two [T, C] id arrays (None if equal prefix and shape)."""
    n = min(len(out_a), len(out_b))
    d = np.nonzero((out_a[:n] != out_b[:n]).any(axis=1))[0]
    if d.size:
        return int(d[0])
    return None if len(out_a) == len(out_b) else n
