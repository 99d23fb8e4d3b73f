"""Utilities: shapes, dtypes, logging/metrics."""
