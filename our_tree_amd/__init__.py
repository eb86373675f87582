"""our_tree_amd -- MI355X (gfx950)-native bulk symmetric-cipher engine.

Same capabilities as the reference maleiwhat/Our-Tree (AES-128/192/256
ECB/CBC/CFB128/CTR, ARC4/RC4, thread/device scaling harnesses, results.* logs),
re-designed for MI355X: hand-written HIP kernels (LDS T-table, bitsliced VALU,
many-stream RC4), a pinned multi-stream host pipeline, and data parallelism
over RCCL/xGMI.  See SURVEY.md for the component map and docs/ for design notes.

Sub-packages:
    models   -- cipher families (AES, ARC4, RC4MultiStream) + CPU oracle
    ops      -- device ops on torch tensors (native gfx950 kernels)
    parallel -- shard planner, torch.distributed DP, host streaming engine
    utils    -- results formats, timing, device info
"""
__version__ = "0.1.0"

from . import _native  # noqa: F401
