"""Utilities: tagged logging, metrics CSV, plots, checkpoints, timers, fault injection, profiling."""
