"""mlapi_amd — an MI355X-native ML-inference microservice framework.

Capabilities of achbogga/mlAPI (FastAPI ``/predict`` + ``/files/`` over a pickled sklearn
LogisticRegression) re-designed for AMD Instinct MI355X (gfx950): hand-written HIP kernels for the
model math, a native C++ batching engine and HTTP front end, RCCL data-parallel replicas.
"""
__version__ = "0.1.0"
