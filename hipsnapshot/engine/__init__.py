"""Execution engine: memory-budgeted pipelines, device staging, HBM freeze."""
