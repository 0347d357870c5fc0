"""Python binding + tooling of the MI355X SMEM seeding engine (libsmemgpu.so)."""
from .lib import (Batch, Gpu, Index, SA, Options, Results, SmemError, aln_opt, build_id, device_count, kernel_id, load,
                  seed, source_hash)  # noqa: F401
