"""Prometheus metrics: registry (prom-client semantics), default process metrics, HTTP exposer."""
from .registry import Counter, Gauge, Histogram, NativeHistogramView, Registry, parse_exposition  # noqa: F401
from .server import MetricsServer  # noqa: F401
from .process import default_metrics  # noqa: F401
