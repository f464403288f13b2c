"""The reference's parity gate -- drop-in for utils/test_utils.py:4-8."""
import torch


def allclose(a, b, atol_ratio=0.01):
    """torch.allclose(a, b, atol=atol_ratio * max|b|) (rtol 1e-5); False when max|b| is NaN."""
    mb = torch.max(torch.abs(b))
    if torch.isnan(mb):
        return False
    return torch.allclose(a, b, atol=float(atol_ratio * mb))
