"""Utilities: config reader, metrics, timers."""
