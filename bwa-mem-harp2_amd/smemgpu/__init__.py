"""Python binding + tooling of the MI355X SMEM seeding engine (libsmemgpu.so)."""
from .lib import (Batch, Gpu, Index, SA, Options, Results, SmemError, device_count, load, seed)  # noqa: F401
