"""Serving: batching engine client, checkpoint hot-reload, native HTTP server, DP replicas."""
