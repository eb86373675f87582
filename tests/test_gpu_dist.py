"""The RCCL (torch.distributed backend "nccl") code path on a real MI355X.

Multi-rank RCCL needs one GPU per rank, so on the one-GPU test box this runs a
world-size-1 RCCL group in-process: ScatterGatherPipeline issues the same
RCCL scatter / async gather on its two extra communicators as at 8 ranks, and
allreduce_max runs an RCCL all-reduce on a device tensor.  Results are checked
against the CPU oracle.  Multi-rank correctness is covered by
tests/test_dist_cpu.py (gloo, world sizes 2 and 3)."""
import os

import pytest
import torch

from our_tree_amd.models import cpu_ref

pytestmark = pytest.mark.gpu


def test_rccl_scatter_gather_pipeline(gpu, rccl_world1):
    pdist = rccl_world1
    import torch.distributed as dist

    assert dist.get_backend() == "nccl"
    key, ctr0 = os.urandom(16), (2**64 - 7).to_bytes(16, "big")
    n = (3 << 20) + 37  # 4 rounds of 1 MiB, uneven tail
    g = torch.Generator().manual_seed(3)
    full = torch.randint(0, 256, (n,), dtype=torch.uint8, generator=g).to(gpu)
    exp = cpu_ref.ctr(key, ctr0, full.cpu().numpy().tobytes())
    for overlap in (True, False):
        res = pdist.scatter_ctr(full, n, key, ctr0, chunk_per_rank=1 << 20, overlap=overlap)
        torch.cuda.synchronize()
        assert res.device.type == "cuda"
        assert res.cpu().numpy().tobytes() == exp, f"overlap={overlap}"
    pipe = pdist.ScatterGatherPipeline(1 << 16, device=gpu)
    assert pipe.comm and pipe.overlap and pipe.g_sc is not None
    assert pdist.allreduce_max(2.5) == 2.5


def test_rccl_sharded_cbc_decrypt(gpu, rccl_world1):
    pdist = rccl_world1
    key, iv = os.urandom(32), os.urandom(16)
    pt = os.urandom(16 * 5000)
    ct = torch.frombuffer(bytearray(cpu_ref.cbc(key, iv, pt)), dtype=torch.uint8).to(gpu)
    out = pdist.cbc_decrypt_sharded(ct, key, iv)
    torch.cuda.synchronize()
    assert out.cpu().numpy().tobytes() == pt
    loc = torch.frombuffer(bytearray(pt), dtype=torch.uint8).to(gpu)
    ctr0 = os.urandom(16)
    pdist.sharded_ctr_(loc, key[:16], ctr0)
    torch.cuda.synchronize()
    assert loc.cpu().numpy().tobytes() == cpu_ref.ctr(key[:16], ctr0, pt)


def test_multi_gpu_api_matrix(gpu, rccl_world1, monkeypatch):
    """One shared matrix over every multi-GPU entry point: the same stream,
    key and counter/IV through the single-process C++ paths (otc_multi_run
    direct with 1 and 3 logical shards, otc_multi_run over RCCL,
    otc_multi_ctr_resident) and the one-process-per-GPU torch.distributed
    paths (sharded_ctr_, scatter_ctr over several scatter rounds,
    cbc_decrypt_sharded), against the one-shot device ops and the C oracle.
    The semantics table is in docs/COMPONENTS.md (2.5)."""
    import numpy as np

    from our_tree_amd import ops
    from our_tree_amd.parallel import stream as pstream

    pdist = rccl_world1
    monkeypatch.setenv("OTC_SHARE_GPUS", "1")
    key, iv = os.urandom(16), (2**64 - 300).to_bytes(16, "big")  # crosses the 64-bit carry
    n = (3 << 20) + 16 * 11
    x = np.random.default_rng(11).integers(0, 256, n, dtype=np.uint8)
    want = {"ctr": cpu_ref.ctr(key, iv, x.tobytes()), "cbc-dec": cpu_ref.cbc(key, iv, x.tobytes(), decrypt=True)}
    got = {}
    for mode in ("ctr", "cbc-dec"):
        for name, ngpus, strategy in (("direct1", 1, "direct"), ("direct3", 3, "direct"), ("rccl1", 1, "rccl")):
            xp, y = pstream.pinned_empty(n), pstream.pinned_empty(n)  # pinned: the RCCL job's root copies overlap
            xp[:] = x
            pstream.multi_gpu_run(mode, xp, y, key, iv, ngpus=ngpus, strategy=strategy, chunk_bytes=256 << 10)
            got[(mode, "otc_multi_run/" + name)] = y.tobytes()
    t = torch.from_numpy(x.copy()).to(gpu)
    r = t.clone()
    pstream.multi_ctr_resident([r], key, iv)
    got[("ctr", "otc_multi_ctr_resident")] = r.cpu().numpy().tobytes()
    r = t.clone()
    pdist.sharded_ctr_(r, key, iv)
    got[("ctr", "dist.sharded_ctr_")] = r.cpu().numpy().tobytes()
    got[("ctr", "dist.scatter_ctr")] = pdist.scatter_ctr(t, n, key, iv, chunk_per_rank=1 << 20).cpu().numpy().tobytes()
    got[("cbc-dec", "dist.cbc_decrypt_sharded")] = pdist.cbc_decrypt_sharded(t, key, iv).cpu().numpy().tobytes()
    got[("ctr", "ops.ctr")] = ops.ctr(t, key, iv).cpu().numpy().tobytes()
    got[("cbc-dec", "ops.cbc_decrypt")] = ops.cbc_decrypt(t, key, iv).cpu().numpy().tobytes()
    torch.cuda.synchronize()
    bad = [k for k, v in got.items() if v != want[k[0]]]
    assert not bad, bad
    assert len(got) == 12
