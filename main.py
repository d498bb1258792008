"""ASGI entry point with the reference's name: `uvicorn main:app` (reference README.md:16).

The app is mlapi_amd's FastAPI app: same routes, schemas and responses as the reference
`main.py`, with the model served by the batching engine (HIP kernels on MI355X, or the C++ CPU
backend when no GPU is visible). For the native high-throughput front end use
`python -m mlapi_amd.serve`.
"""
from mlapi_amd.api.app import create_app

app = create_app()
