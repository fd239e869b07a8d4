"""Shared utilities (audio I/O, ...)."""
