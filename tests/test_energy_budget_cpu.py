"""tools/energy_budget.py on the built headline kernel (docs/PERF.md round 6):
the instruction mix is read from the gfx950 code object, the parts of the
budget add up to the measured J/GB, and the S-box / MixColumns circuit is
the largest part -- the finding that pointed the round's energy work at the
memory system (the one reducible term outside the circuit)."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
OBJ = os.path.join(ROOT, "build", "obj", "hip", "aes_bs.o")
LLVM = "/opt/rocm/lib/llvm/bin"


@pytest.fixture(scope="module")
def eb():
    if not os.path.exists(OBJ) or not os.path.exists(f"{LLVM}/clang-offload-bundler"):
        pytest.skip("no built objects (make) or no ROCm LLVM tools")
    sys.path.insert(0, os.path.join(ROOT, "tools"))
    import energy_budget

    return energy_budget


def test_budget_closes_and_circuit_dominates(eb):
    name, mix = eb.kernel_mix(OBJ, r"k_aes_bs_t3ILi10ELi0ELi8ELb1ELb1E")
    assert "k_aes_bs_t3" in name
    # the AES-128 CTR bulk task: ~12.8k VALU (docs/PERF.md round 3), 32
    # ciphertext stores, 8 LDS-DMA plaintext loads, no scratch
    valu = sum(v for k, v in mix.items() if k.startswith("v_"))
    assert 12000 < valu < 13800, valu
    assert mix["vmem_store"] == 32 and mix["vmem_load_lds"] == 8
    b = eb.budget(mix, jgb=0.808, gbps=1702.4, idle_w=264.0, hbm_pj_per_bit=4.0)
    total = sum(r["jgb_scaled"] for r in b["rows"])
    assert abs(total - 0.808) < 1e-3, total
    shares = {r["part"].split(" (")[0]: r["share"] for r in b["rows"]}
    circuit = next(v for k, v in shares.items() if k.startswith("S-box"))
    assert circuit == max(shares.values()) and circuit > 0.5, shares


def test_classifier_forms(eb):
    assert eb.classify("v_bitop3_b32", "v1, v2, v3, v4 bitop3:0x96") == "v_bitop3_vvv"
    assert eb.classify("v_bitop3_b32", "v1, s4, v3, v4 bitop3:0x96") == "v_bitop3_vvs"
    assert eb.classify("v_xor_b32_e32", "v1, v2, v3") == "v_xor"
    assert eb.classify("global_store_dwordx4", "v12, v[148:151], s[2:3] nt") == "vmem_store"
    assert eb.classify("global_load_lds_dwordx4", "v12, s[26:27] nt") == "vmem_load_lds"
    assert eb.classify("s_waitcnt", "vmcnt(0)") == "wait_nop"
