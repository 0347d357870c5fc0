"""Python binding + tooling of the MI355X SMEM seeding engine (libsmemgpu.so)."""
from .lib import (Batch, Gpu, Index, SA, Options, Results, SmemError, build_id, device_count, load, seed,
                  source_hash)  # noqa: F401
