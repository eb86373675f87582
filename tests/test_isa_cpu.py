"""Static guards on the built gfx950 code (no GPU needed): the bitsliced bulk
kernels stay spill-free and within their VALU budget per 2048-block task
(tools/isa_count.py; profiles/r3/sbox77: 12,802 AES-128, 18,610 AES-256 --
the counts rocprofv3 measures, profiles/r3/sbox79/pmc_ctr128_bulk.txt).  A
register-pressure regression shows up here as scratch > 0 long before a GPU
run, and a lost optimisation as a VALU jump."""
import os
import re
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj", "hip", "aes_bs.o")
LLVM = "/opt/rocm/lib/llvm/bin"

BUDGET = {("CTR", "AES-128"): 12900, ("CTR", "AES-192"): 15800, ("CTR", "AES-256"): 18700}


@pytest.fixture(scope="module")
def counts():
    if not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built aes_bs.o (make) or no ROCm LLVM tools")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_count.py"), OBJ], check=True,
                         capture_output=True, text=True).stdout
    rows = {}
    for line in out.splitlines():
        m = re.search(r": ([\w-]+) (AES-\d+) VALU (\d+) .* VGPRs (-?\d+) scratch (-?\d+) scratch_ops (\d+)", line)
        if m:
            rows[(m.group(1), m.group(2))] = (int(m.group(3)), int(m.group(4)), int(m.group(5)), int(m.group(6)))
    return rows


def test_every_bulk_kernel_found(counts):
    """CTR has a bulk launch; ECB and the decryptions run only as claim
    kernels (beside the T-table, or alone for impl "bitslice")."""
    for mode in ("CTR", "ECB-claim", "ECB-dec-claim", "CBC-dec-claim", "CFB-dec-claim"):
        for bits in ("AES-128", "AES-192", "AES-256"):
            assert (mode, bits) in counts, (mode, bits, sorted(counts))
    assert not any(k[0] in ("ECB", "ECB-dec", "CBC-dec", "CFB-dec") for k in counts), sorted(counts)


def test_bulk_kernels_spill_free(counts):
    """Encryption kernels (CFB decryption runs the forward cipher): no scratch
    at all.  The inverse-cipher kernels (L o
    InvMixColumns o L is 125 nodes per column against MixColumns' 55) keep a
    few 64-bit addresses in scratch across the rounds: at most 28 scratch
    instructions per 2048-block task (beside ~26k VALU; the split's claim
    loop adds a few), none in the rounds themselves."""
    for key, (valu, vgprs, scratch, sops) in counts.items():
        if key[0].startswith("CBC-dec-seg"):
            assert sops <= 40, (key, sops)  # + the segment-IV blend in the output phase
        elif key[0].startswith(("ECB-dec", "CBC-dec")):
            assert sops <= 28, (key, sops)
        else:
            assert scratch == 0, (key, scratch)
        assert 0 < vgprs <= 168, (key, vgprs)  # 3 waves per SIMD


def test_claim_kernels_fit_beside_ttable(counts):
    """The split's bitsliced claim kernels (one task per loop trip) exist for
    every split mode, and one wave of each fits in a SIMD's 512 registers
    beside the 4 waves of the T-table claim kernel (ECB: 88 allocated each, so
    <= 160; the others: <= 168 beside 4 x 64-72)."""
    for mode in ("ECB-claim", "ECB-dec-claim", "CBC-dec-claim", "CFB-dec-claim", "CBC-dec-seg-claim",
                 "CFB-dec-seg-claim"):
        for bits in ("AES-128", "AES-192", "AES-256"):
            valu, vgprs, scratch, sops = counts[(mode, bits)]
            assert vgprs <= (160 if mode == "ECB-claim" else 168), (mode, bits, vgprs)


def test_ctr_valu_budget(counts):
    for key, budget in BUDGET.items():
        assert counts[key][0] <= budget, (key, counts[key][0], budget)


def test_split_pairs_share_a_simd():
    """Co-residency of the claimed split, from the code objects: for every
    split mode, 4 waves of the T-table claim kernel plus 1 wave of the
    bitsliced claim kernel fit in a SIMD's 512 registers, counted as the
    kernel descriptors allocate them (8-register granules; hipcc pads a
    static-LDS kernel's descriptor to its LDS occupancy, which made the
    round-4 "split" run its halves one after the other, docs/PERF.md round 5)
    -- a T-table change that adds a few registers would silently turn the
    split into time slicing."""
    tt_obj = os.path.join(ROOT, "build", "obj", "hip", "aes_tt.o")
    if not os.path.exists(tt_obj) or not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built objects (make) or no ROCm LLVM tools")
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_count

    def vgprs(obj):
        with tempfile.TemporaryDirectory() as tmp:
            return isa_count.descriptor_vgprs(isa_count.code_object(obj, tmp))

    tt, bs = vgprs(tt_obj), vgprs(OBJ)
    alloc = lambda n: -(-n // 8) * 8
    # split mode: (T-table claim kernel name part, bitsliced claim mode number)
    pairs = {"ECB": ("k_aes_ecb_tt_claim", 1), "ECB-dec": ("k_aes_dec_tt_claimILi{nr}ELi0E", 2),
             "CBC-dec": ("k_aes_dec_tt_claimILi{nr}ELi1E", 3), "CFB-dec": ("k_aes_cfb_tt_claim", 4),
             "CBC-dec-seg": ("k_aes_dec_tt_claimILi{nr}ELi2E", 5), "CFB-dec-seg": ("k_aes_cfbseg_tt_claim", 6)}
    seen = 0
    for mode, (tpat, bmode) in pairs.items():
        for nr in (10, 12, 14):
            tnames = [k for k in tt if tpat.format(nr=nr) in k and f"ILi{nr}E" in k]
            bnames = [k for k in bs if f"k_aes_bs_claimILi{nr}ELi{bmode}E" in k]
            assert tnames and bnames, (mode, nr)
            t, b = max(tt[k] for k in tnames), max(bs[k] for k in bnames)
            assert 4 * alloc(t) + alloc(b) <= 512, (mode, nr, t, b)
            seen += 1
    assert seen == 18


def _vgprs(obj):
    """kernel -> (descriptor VGPRs, scratch bytes)"""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_count

    with tempfile.TemporaryDirectory() as tmp:
        co = isa_count.code_object(obj, tmp)
        meta, desc = isa_count.metadata(co), isa_count.descriptor_vgprs(co)
    return {k: (v, meta.get(k + ".kd", meta.get(k, (0, -1)))[1]) for k, v in desc.items()}


def test_descriptors_match_register_use():
    """Every claim kernel's descriptor allocates what the kernel uses (the
    metadata's .vgpr_count rounded to the granule), not an occupancy-padded
    count: the padding is what kept the round-4 split from co-running."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_count

    objs = [os.path.join(ROOT, "build", "obj", "hip", f"{o}.o") for o in ("aes_tt", "aes_bs")]
    if not all(os.path.exists(o) for o in objs) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built objects (make) or no ROCm LLVM tools")
    seen = 0
    for obj in objs:
        with tempfile.TemporaryDirectory() as tmp:
            co = isa_count.code_object(obj, tmp)
            meta, desc = isa_count.metadata(co), isa_count.descriptor_vgprs(co)
        for k, v in desc.items():
            if "claim" in k:
                used = meta.get(k + ".kd", meta.get(k))[0]
                assert v == -(-used // 8) * 8, (k, v, used)
                seen += 1
    assert seen >= 30


def test_ttable_claim_kernels_have_no_static_lds():
    """The T-table claim kernels address their dynamic-LDS tables by integer
    from address 0 (aes_tt.hip DynTbl): that holds only while they declare no
    static LDS, i.e. their descriptors' fixed group segment is 0 bytes."""
    import tempfile

    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import isa_count

    tt_obj = os.path.join(ROOT, "build", "obj", "hip", "aes_tt.o")
    if not os.path.exists(tt_obj) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built aes_tt.o (make) or no ROCm LLVM tools")
    with tempfile.TemporaryDirectory() as tmp:
        d = isa_count.descriptor_vgprs(isa_count.code_object(tt_obj, tmp), with_lds=True)
    claims = {k: v for k, v in d.items() if "_claim" in k}
    assert len(claims) >= 24, sorted(claims)
    for k, (vg, lds) in claims.items():
        assert lds == 0, (k, lds)
    # the grid kernels keep their static tables (128 / 160 KiB)
    assert any(lds >= 128 << 10 for k, (vg, lds) in d.items() if "_claim" not in k)


def test_operand_statistics_as_documented():
    """The static operand facts docs/PERF.md (round 6, "three hypotheses")
    prices with tools/ubench/valu_bank.hip: ~17% of the AES-128 CTR bulk
    kernel's VALU read an SGPR (a stream costs extra only when most of its
    instructions do), and 6,078 of its 9,476 three-VGPR v_bitop3 share a
    register bank (tools/isa_operands.py)."""
    if not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built aes_bs.o (make) or no ROCm LLVM tools")
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "isa_operands.py"), OBJ], check=True,
                         capture_output=True, text=True).stdout
    m = re.search(r"VALU (\d+), reading an SGPR (\d+)", out)
    assert m, out
    valu, sg = int(m.group(1)), int(m.group(2))
    assert 12000 <= valu <= 12900 and 0.10 <= sg / valu <= 0.25, (valu, sg)
    three = {int(k): int(v) for k, v in re.findall(r"\('bitop3', 3, (\d)\): (\d+)", out)}
    assert sum(three.values()) > 8000 and 0.4 <= (three.get(1, 0) + three.get(2, 0)) / sum(three.values()) <= 0.8
