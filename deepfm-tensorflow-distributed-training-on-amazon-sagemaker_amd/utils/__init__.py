"""Auxiliary subsystems: profiling/tracing, failure detection, fault injection,
numerics checks."""
