"""Vendor Specific Plugins: mock, GPU (MI355X data plane), and the OvS/P4-style vendors re-expressed on it."""
from .base import MockVsp, VspBase  # noqa: F401
