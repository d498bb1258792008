"""Data parallelism over RCCL/xGMI: process groups, collectives, DP serving and DP training."""
