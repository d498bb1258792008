"""Config, metrics, logging helpers."""
