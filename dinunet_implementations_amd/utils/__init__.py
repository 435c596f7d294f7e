"""Utilities: metrics, logging, checkpoints, timing."""
