"""TEST INFRASTRUCTURE ONLY — the CPU oracle for the SkeletonDiffusion sampling hot path.

Only `tests/`, `__graft_entry__.smoke()` and `bench.py`'s `cpu_baseline` leg may import this
package, and only as the checker / CPU baseline.  The product (`skeletondiffusion_amd`) never
imports it: its sampling path is the HIP library and fails loudly when that is missing.
"""
from .skeldiff_oracle import *  # noqa: F401,F403
