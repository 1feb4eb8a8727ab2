"""Utilities: test helpers, RSS profiler, roctx tracing."""
