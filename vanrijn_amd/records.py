"""Device accumulation records (include/vanrijn_amd.h, ABI 7), for numpy arrays and torch tensors.

A tile of n pixels has 8 n doubles of records in two halves (row-major pixels):

    state[0 : 4n]  = n x {sum X, sum Y, sum Z, weight}        colour_sum, weight
    state[4n : 8n] = n x {bias X, bias Y, bias Z, weight bias} Kahan compensations

(AccumulationBuffer's colour_sum / colour_bias / weight / weight_bias, accumulation_buffer.rs:6-12,
44-60).  The first half is the merge-exact part: adding it merges disjoint sample sets the way
merge_tile's weighted blend does (accumulation_buffer.rs:62-85), so the cross-GPU reduce is one
in-place collective over a contiguous 32 B per pixel (vanrijn_amd/distributed.py).
"""
import numpy as np

RECORD = 8  # f64 per pixel
SUMS = 4    # f64 per pixel in the merge-exact half


def pixels(state):
    n = state.numel() if hasattr(state, "numel") else state.size
    if n % RECORD:
        raise ValueError(f"{n} doubles are not whole records of {RECORD}")
    return n // RECORD


def sums(state):
    """[n, 4] view of {sum X, sum Y, sum Z, weight} (flat state, numpy or torch)."""
    n = pixels(state)
    return state.reshape(-1)[:SUMS * n].reshape(n, SUMS)


def compensations(state):
    """[n, 4] view of the Kahan compensations {bias X, bias Y, bias Z, weight bias}."""
    n = pixels(state)
    return state.reshape(-1)[SUMS * n:].reshape(n, SUMS)


def fields(state, shape=None):
    """numpy copies of the AccumulationBuffer arrays: colour_sum, colour_bias [.., 3], weight,
    weight_bias [..]; `shape` = (height, width) reshapes the pixel axis."""
    s = np.asarray(state.cpu() if hasattr(state, "cpu") else state, dtype=np.float64)
    a, b = sums(s), compensations(s)
    out = {"colour_sum": a[:, 0:3].copy(), "colour_bias": b[:, 0:3].copy(), "weight": a[:, 3].copy(),
           "weight_bias": b[:, 3].copy()}
    if shape is not None:
        out = {k: v.reshape(tuple(shape) + v.shape[1:]) for k, v in out.items()}
    return out


def from_fields(colour_sum, colour_bias, weight, weight_bias):
    """Flat numpy records from the four AccumulationBuffer arrays (any pixel shape)."""
    cs = np.asarray(colour_sum, dtype=np.float64).reshape(-1, 3)
    n = len(cs)
    out = np.empty(RECORD * n)
    a, b = out[:SUMS * n].reshape(n, SUMS), out[SUMS * n:].reshape(n, SUMS)
    a[:, 0:3] = cs
    a[:, 3] = np.asarray(weight, dtype=np.float64).reshape(-1)
    b[:, 0:3] = np.asarray(colour_bias, dtype=np.float64).reshape(-1, 3)
    b[:, 3] = np.asarray(weight_bias, dtype=np.float64).reshape(-1)
    return out
