"""Command-line front end:  python -m our_tree_amd <command> ...

  info                         device(s), CUs, clock, native build
  selftest [--gpu]             FIPS-197 / SP 800-38A / RFC 3686 / ARC4 known-answer
                               tests on the C oracle; --gpu: the same vectors through
                               the gfx950 kernels
  crypt SRC DST --key HEX [--iv HEX] [--mode ctr|ecb|cbc-dec]
        [--chunk 256M] [--cpu] resumable file-to-file job (parallel/filejob.py:
                               pinned 3-stream GPU pipeline, JSON resume cursor
                               next to DST; re-run the same command to resume)

The reference's only interfaces were its benchmark binaries
(/root/reference/test.c, aes-modes/test.c, aes-gpu/Source/main_ecb_[ed].cu);
those live on as bin/test, bin/aes_test, bin/aes_ecb_e, bin/aes_ecb_d.
"""
from __future__ import annotations

import argparse
import json
import sys


def _size(s: str) -> int:
    mult = {"K": 1 << 10, "M": 1 << 20, "G": 1 << 30}
    s = s.strip().upper()
    return int(float(s[:-1]) * mult[s[-1]]) if s and s[-1] in mult else int(s)


def cmd_info(_args) -> int:
    from . import _native

    out = {"native_gpu_lib": _native.gpu_lib_available()}
    try:
        import torch

        out["torch"] = torch.__version__
        out["gpus"] = torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception as e:  # pragma: no cover
        out["torch_error"] = repr(e)
    if out["native_gpu_lib"] and out.get("gpus"):
        lib = _native.require_gpu_lib()
        out["build"] = lib.otc_build_info().decode()
        out["devices"] = [{"cus": lib.otc_device_cus(d), "peak_clock_mhz": lib.otc_device_clock_khz(d) // 1000}
                          for d in range(lib.otc_device_count())]
    print(json.dumps(out, indent=1))
    return 0


# FIPS-197 appendix C.1 / C.3 and SP 800-38A F.5.1 (CTR-AES128.Encrypt, block 1)
_KATS = [
    ("ecb", "000102030405060708090a0b0c0d0e0f", "", "00112233445566778899aabbccddeeff",
     "69c4e0d86a7b0430d8cdb78070b4c55a"),
    ("ecb", "000102030405060708090a0b0c0d0e0f101112131415161718191a1b1c1d1e1f", "",
     "00112233445566778899aabbccddeeff", "8ea2b7ca516745bfeafc49904b496089"),
    ("ctr", "2b7e151628aed2a6abf7158809cf4f3c", "f0f1f2f3f4f5f6f7f8f9fafbfcfdfeff",
     "6bc1bee22e409f96e93d7e117393172a", "874d6191b620e3261bef6864990db6ce"),
]


def cmd_selftest(args) -> int:
    from .models import cpu_ref

    res = cpu_ref.self_tests(1)
    ok = all(v == 0 for v in res.values())
    print(json.dumps({"cpu_oracle_self_tests": res}))
    if args.gpu:
        import torch

        from . import ops

        for mode, key, iv, pt, ct in _KATS:
            k, x = bytes.fromhex(key), torch.tensor(list(bytes.fromhex(pt)), dtype=torch.uint8, device="cuda")
            y = ops.ecb_encrypt(x, k) if mode == "ecb" else ops.ctr(x, k, bytes.fromhex(iv))
            good = y.cpu().numpy().tobytes().hex() == ct
            ok = ok and good
            print(json.dumps({"gpu_kat": mode, "key_bits": len(k) * 8, "ok": good}))
    return 0 if ok else 1


def cmd_crypt(args) -> int:
    from .parallel import filejob

    key = bytes.fromhex(args.key)
    iv = bytes.fromhex(args.iv) if args.iv else bytes(16)
    if len(key) not in (16, 24, 32) or len(iv) != 16:
        print("key must be 16/24/32 bytes and iv 16 bytes (hex)", file=sys.stderr)
        return 2
    backend = filejob.cpu_backend() if args.cpu else filejob.gpu_backend(chunk_bytes=_size(args.chunk))
    r = filejob.crypt_file(args.src, args.dst, key, iv, mode=args.mode, chunk_bytes=_size(args.chunk),
                           backend=backend)
    print(json.dumps(r))
    return 0 if r.get("done") else 1


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="python -m our_tree_amd", description=__doc__.split("\n")[0])
    sub = ap.add_subparsers(dest="cmd", required=True)
    sub.add_parser("info").set_defaults(fn=cmd_info)
    st = sub.add_parser("selftest")
    st.add_argument("--gpu", action="store_true")
    st.set_defaults(fn=cmd_selftest)
    cr = sub.add_parser("crypt")
    cr.add_argument("src")
    cr.add_argument("dst")
    cr.add_argument("--key", required=True, help="hex")
    cr.add_argument("--iv", default="", help="hex IV / initial counter block (16 bytes)")
    cr.add_argument("--mode", default="ctr", choices=["ctr", "ecb", "cbc-dec"])
    cr.add_argument("--chunk", default="256M")
    cr.add_argument("--cpu", action="store_true", help="C-oracle backend (no GPU)")
    cr.set_defaults(fn=cmd_crypt)
    args = ap.parse_args(argv)
    return args.fn(args)


if __name__ == "__main__":
    sys.exit(main())
