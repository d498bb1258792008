"""Model IR (linear / logistic / softmax regression) and the sklearn-compatible estimator."""
from mlapi_amd.models.linear import Kind, LinearModel

__all__ = ["Kind", "LinearModel"]
