"""Packaging: ``pip install .`` (or ``pip install -e .``) builds the gfx950 extension with hipcc
(mlapi_amd/_build.py) and installs the ``mlapi_amd`` package plus the reference-compatible
``main.py`` entry module (``uvicorn main:app``).

The reference pins its environment in requirements.txt (`requirements.txt:1-17`); the runtime
requirements here are declared below and mirrored in requirements.txt. Metadata lives in this file
(not in a PEP 621 table) so that the setuptools shipped with the ROCm images (59.x) reads it.
"""
import os
import sys

from setuptools import find_packages, setup
from setuptools.command.build_py import build_py

HERE = os.path.dirname(os.path.abspath(__file__))


class BuildWithHip(build_py):
    """Compile csrc/ for gfx950 into mlapi_amd/_C*.so before the package files are copied."""

    def run(self):
        sys.path.insert(0, HERE)
        from mlapi_amd import _build

        _build.build(verbose=True)
        super().run()


setup(
    name="mlapi-amd",
    version="0.1.0",
    description=("MI355X-native ML-inference microservice: FastAPI-compatible /predict over sklearn "
                 "LogisticRegression checkpoints, batched gfx950 HIP kernels, RCCL data parallelism"),
    license="MIT",
    license_files=["LICENSE"],
    python_requires=">=3.10",
    packages=find_packages(include=["mlapi_amd", "mlapi_amd.*"]),
    py_modules=["main"],
    package_data={"mlapi_amd": ["_C*.so", "bin/mlapi-loadgen"]},
    # torch must be a ROCm build (the extension binds to the HIP runtime torch loads);
    # python-multipart is not needed (mlapi_amd.api.multipart replaces it).
    install_requires=["torch>=2.4", "numpy>=1.20", "fastapi>=0.63", "pydantic>=1.7", "uvicorn>=0.13",
                      "pandas>=1.2"],
    extras_require={
        "train": ["scipy>=1.6", "scikit-learn>=0.24"],
        "metrics": ["prometheus_client>=0.9"],
        "test": ["pytest>=7", "pytest-timeout", "httpx", "hypothesis", "scikit-learn>=0.24", "scipy>=1.6"],
    },
    entry_points={"console_scripts": [
        "mlapi-serve = mlapi_amd.serve.__main__:main",
        "mlapi-train = mlapi_amd.train.__main__:main",
        "mlapi-launch = mlapi_amd.launch:main",
    ]},
    cmdclass={"build_py": BuildWithHip},
)
