"""Concurrency / scale-out: per-key ordering and multi-process competing consumers."""
from .ordering import KeyedSerializer  # noqa: F401
