#!/usr/bin/env python3
"""Static instruction counts of the bitsliced bulk kernels in a built object.

Extracts the gfx950 code object from a hipcc object's .hip_fatbin section
(llvm-objcopy + clang-offload-bundler), disassembles it and prints, for every
k_aes_bs_t3 instantiation compiled for full tasks only (the bulk launch: one
2048-block task per wave, straight-line code), the VALU / SALU / SMEM /
vector-memory instruction counts, VGPRs and scratch bytes, and the same for
the split's claim kernels (MODE-claim: one task per loop trip) (CTR-nocache: the
kernel CTR falls back to when its counter-caching tables cannot be allocated).  The kernel has no
loops, so the static VALU count is the VALU per task that rocprofv3's
SQ_INSTS_VALU / SQ_WAVES reports (profiles/r3/sbox79: 13,058 vs 13,056.5).

    tools/isa_count.py build/obj/hip/aes_bs.o [build/obj-VARIANT/hip/aes_bs.o ...]
"""
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
NAMES = {"Li10E": "AES-128", "Li12E": "AES-192", "Li14E": "AES-256"}


def code_object(obj, tmp):
    fat = os.path.join(tmp, "fatbin")
    co = os.path.join(tmp, "co")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "o")],
                   check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--targets={TARGET}",
                    f"--input={fat}", f"--output={co}"], check=True)
    return co


def metadata(co):
    """kernel symbol -> (vgpr_count, private_segment_fixed_size) from the notes"""
    notes = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                           text=True).stdout
    out = {}
    for blk in notes.split("  - .agpr_count:")[1:]:
        name = re.search(r"\.name:\s+(\S+)", blk)
        vg = re.search(r"\.vgpr_count:\s+(\d+)", blk)
        pr = re.search(r"\.private_segment_fixed_size:\s+(\d+)", blk)
        if name:
            out[name.group(1)] = (int(vg.group(1)) if vg else -1, int(pr.group(1)) if pr else -1)
    return out


def descriptor_vgprs(co, with_lds=False):
    """kernel symbol -> VGPRs the hardware allocates per wave, from the kernel
    descriptor (compute_pgm_rsrc1 bits 5:0 = granules of 8 minus 1 on gfx950
    wave64).  This, not the metadata's .vgpr_count, decides co-residency: with
    a static LDS array hipcc pads the descriptor up to the occupancy the LDS
    allows (csrc/hip/aes_tt.hip tt_lds).  with_lds: (VGPRs, the descriptor's
    group_segment_fixed_size = static LDS bytes)."""
    secs = subprocess.run([f"{LLVM}/llvm-readelf", "-S", "-W", co], check=True, capture_output=True,
                          text=True).stdout
    layout = []  # (addr, file offset, size)
    for m in re.finditer(r"\]\s+\S+\s+\S+\s+([0-9a-f]{8,})\s+([0-9a-f]{6,})\s+([0-9a-f]{6,})", secs):
        layout.append((int(m.group(1), 16), int(m.group(2), 16), int(m.group(3), 16)))
    syms = subprocess.run([f"{LLVM}/llvm-readelf", "-s", "-W", co], check=True, capture_output=True,
                          text=True).stdout
    data = open(co, "rb").read()
    out = {}
    for m in re.finditer(r"^\s*\d+:\s+([0-9a-f]+)\s+64\s+OBJECT\s+\S+\s+\S+\s+\S+\s+(\S+)\.kd$", syms, re.M):
        addr = int(m.group(1), 16)
        for a, off, size in layout:
            if a <= addr < a + size:
                rsrc1 = int.from_bytes(data[addr - a + off + 48:addr - a + off + 52], "little")
                lds = int.from_bytes(data[addr - a + off:addr - a + off + 4], "little")
                out[m.group(2)] = (((rsrc1 & 0x3F) + 1) * 8, lds) if with_lds else ((rsrc1 & 0x3F) + 1) * 8
                break
    return out


def main():
    for obj in sys.argv[1:]:
        with tempfile.TemporaryDirectory() as tmp:
            co = code_object(obj, tmp)
            asm = subprocess.run([f"{LLVM}/llvm-objdump", "-d", co], check=True, capture_output=True,
                                 text=True).stdout
            meta = metadata(co)
        for f in re.split(r"\n(?=[0-9a-f]+ <)", asm):
            m = re.match(r"[0-9a-f]+ <(.*?)>:", f)
            if not m:
                continue
            name = m.group(1)
            claim = "k_aes_bs_claim" in name  # the bitsliced half of a claimed split (one loop over tasks)
            if not claim and ("k_aes_bs_t3" not in name or not re.search(r"Lb[01]ELb1EEE", name)):
                continue
            ins = re.findall(r"^\s+([a-z_0-9]+)", f, re.M)
            cnt = lambda p: sum(1 for i in ins if i.startswith(p))
            tm = re.search(r"(?:t3|claim)ILi(\d+)ELi(\d)E", name)
            mode = {"0": "CTR", "1": "ECB", "2": "ECB-dec", "3": "CBC-dec", "4": "CFB-dec", "5": "CBC-dec-seg",
                    "6": "CFB-dec-seg"}.get(tm.group(2), "?") if tm else "?"
            if mode == "CTR" and re.search(r"Lb0ELb1EEE", name):
                mode = "CTR-nocache"  # fallback when the counter-caching tables do not fit
            if claim:
                mode += "-claim"
            bits = NAMES.get(f"Li{tm.group(1)}E", "?") if tm else "?"
            vg, scr = meta.get(name + ".kd", meta.get(name, (-1, -1)))
            print(f"{obj}: {mode} {bits} VALU {cnt('v_')} SALU {cnt('s_') - cnt('s_load') - cnt('s_buffer')} "
                  f"SMEM {cnt('s_load') + cnt('s_buffer')} VMEM {cnt('global_') + cnt('buffer_')} "
                  f"LDS {cnt('ds_')} VGPRs {vg} scratch {scr} scratch_ops {cnt('scratch_')}")


if __name__ == "__main__":
    main()
