"""Utilities: native runtime access, distributed env helpers, logging, checkpointing, profiling."""
