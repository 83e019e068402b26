"""Pins the MFMA accumulation behaviour the rank error bound is derived from."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def test_mfma_probe_model():
    import torch
    from cmve import engine, _lib
    dev = torch.device("cuda", 0)
    out = torch.zeros(10, dtype=torch.float32, device=dev)
    _lib.check(_lib.lib.cmve_mfma_probe(engine.handle(dev), engine._ptr(out)))
    v = out.cpu().numpy().astype(np.float64)
    for f in range(2):  # bf16, f16
        c = v[5 * f: 5 * f + 5]
        # every observed result must lie within the bound's model: at most one fp32 rounding per
        # product (fma chain) -- i.e. |result - exact| <= n_products * 2^-23 * sum|products|
        exact = [1 + 2 ** -21, 1 + 2 ** -23, 1 + 3 * 2 ** -25, 1 + 3 * 2 ** -25, 2 ** -30]
        nprod = [17, 3, 4, 4, 3]
        mag = [1 + 2 ** -21, 1 + 2 ** -23, 1 + 3 * 2 ** -25, 1 + 3 * 2 ** -25, 2 + 2 ** -30]
        for k in range(5):
            assert abs(c[k] - exact[k]) <= nprod[k] * 2 ** -23 * mag[k], (f, k, c[k].hex(), exact[k])
