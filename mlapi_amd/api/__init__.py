"""HTTP API (FastAPI app with the reference's routes, multipart parsing)."""
