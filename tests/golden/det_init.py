"""Deterministic weights for the full-shape parity fixtures (test infrastructure).

The full-size model has 7.5 M parameters: committing its state dict would put 30 MB of
random floats into tests/golden.  Instead the fixture generator (make_golden.py, which runs
the REFERENCE Model3DETR) and the parity tests (which run the product) both overwrite every
parameter and buffer with the same seeded values, keyed by state-dict name, before the
forward.  The values only need the magnitudes of a random init (variance 1/fan_in for the
weights, BatchNorm / LayerNorm affine near (1, 0), fresh running statistics), so activations
and gradients are in the regime the training step starts from.
"""
import zlib

import numpy as np
import torch


def _rs(name, seed):
    return np.random.RandomState((zlib.crc32(name.encode()) + 7919 * seed) % (2 ** 31))


def value(name, shape, seed):
    """float64 array for state-dict entry `name` (product and reference share the key names)."""
    rs = _rs(name, seed)
    leaf = name.rsplit(".", 1)[-1]
    if leaf == "running_mean":
        return np.zeros(shape)
    if leaf == "running_var":
        return np.ones(shape)
    if leaf == "num_batches_tracked":
        return np.zeros(shape)
    if leaf == "gauss_B":                      # position_embedding.py:36-39, gauss_scale 1
        return rs.standard_normal(shape)
    norm = (".bn." in name or ".norm" in name or "norm1" in name or "norm2" in name
            or "norm3" in name or name.startswith("decoder.norm"))
    if len(shape) == 1:
        if norm and leaf == "weight":
            return 1.0 + 0.1 * rs.uniform(-1, 1, shape)
        return 0.05 * rs.uniform(-1, 1, shape)
    fan_in = int(np.prod(shape[1:]))
    b = np.sqrt(3.0 / fan_in)                   # uniform with variance 1 / fan_in
    return rs.uniform(-b, b, shape)


def value32(name, shape, seed):
    """`value` rounded to float32: the product (fp32 parameters) and the float64 reference
    then start from identical numbers"""
    return value(name, shape, seed).astype(np.float32).astype(np.float64)


def probe(name, shape):
    """fixed unit-variance vector per parameter: the fixtures store <grad, probe> for every
    parameter (a sign- and direction-sensitive scalar next to the gradient norm)"""
    return _rs("probe/" + name, 0).standard_normal(shape)


def fill_(module, seed, skip=("mlp_heads.sem_cls_head.weight",)):
    """overwrite every parameter / buffer of `module` (names not in `skip`) in place;
    returns the sorted list of names filled"""
    done = []
    with torch.no_grad():
        for name, t in list(module.state_dict(keep_vars=True).items()):
            if name in skip:
                continue
            v = torch.from_numpy(value32(name, tuple(t.shape), seed))
            t.copy_(v.to(dtype=t.dtype, device=t.device))
            done.append(name)
    return sorted(done)
