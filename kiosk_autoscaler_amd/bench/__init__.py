"""Benchmark harness: Poisson on/off load, reference simulator, metrics (N9)."""
