"""HIP kernel ops (GPU tensors only) and their PyTorch reference oracles."""
