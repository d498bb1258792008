"""Training: exact L-BFGS fit (sklearn parity) and data-parallel mini-batch SGD."""
from mlapi_amd.train.lbfgs import fit_logistic_lbfgs

__all__ = ["fit_logistic_lbfgs"]
