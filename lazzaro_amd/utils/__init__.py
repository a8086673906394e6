"""Utilities: device selection, timers/tracing, logging helpers."""
from .device import default_device, sync  # noqa: F401
