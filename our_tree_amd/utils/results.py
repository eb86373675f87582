"""Result logs: the reference's ``results.*`` line formats (writer + parser)
and a JSON-lines sidecar.

Formats (SURVEY.md section 5 "Metrics / logging"):
* RC4   (test.c:61,84-91,116,125):
  ``RC4, <bytes>, <threads>, \\nGenerated a new key in <us>, \\n<us>, <us>, ...\\n``
* AES CPU (aes-modes/test.c:47,129,209,288): ``<Label>, <bytes>, <threads>, <us>, ...``
* GPU ECB (main_ecb_e.cu:56,62,64): ``AES ECB test, <bytes>: <us>, ...,  Average <us>``
"""
from __future__ import annotations

import json
import re
import statistics


def format_rc4(nbytes: int, threads: int, keygen_us: int, iters_us: list[int]) -> str:
    return (f"RC4, {nbytes}, {threads}, \nGenerated a new key in {keygen_us}, \n"
            + "".join(f"{t}, " for t in iters_us) + "\n")


def format_aes(label: str, nbytes: int, threads: int, iters_us: list[int]) -> str:
    return f"{label}, {nbytes}, {threads}, " + "".join(f"{t}, " for t in iters_us) + "\n"


def format_gpu_ecb(nbytes: int, iters_us: list[int]) -> str:
    avg = sum(iters_us) // max(1, len(iters_us))
    return f"AES ECB test, {nbytes}: " + "".join(f"{t}, " for t in iters_us) + f" Average {avg}\n"


_RC4_HDR = re.compile(r"^RC4, (\d+), (\d+),")
_KEY = re.compile(r"^Generated a new key in (\d+),")
_AES = re.compile(r"^((?:Plain|AESNI|HIP) (?:ECB|CTR|CBC)), (\d+), (\d+), (.*)$")
_GPU = re.compile(r"^AES ECB test, (\d+): (.*?)\s*Average (\d+)")


def _nums(s: str) -> list[int]:
    return [int(x) for x in re.findall(r"\d+", s)]


def parse(text: str) -> list[dict]:
    """Parse any of the three formats into records
    {cipher, label, bytes, threads, keygen_us, us: [...]}."""
    recs, cur = [], None
    lines = text.splitlines()
    for ln in lines:
        ln = ln.rstrip()
        m = _RC4_HDR.match(ln)
        if m:
            cur = {"cipher": "RC4", "label": "RC4", "bytes": int(m[1]), "threads": int(m[2]), "keygen_us": None,
                   "us": _nums(ln[m.end():])}
            recs.append(cur)
            continue
        m = _KEY.match(ln)
        if m and cur is not None:
            cur["keygen_us"] = int(m[1])
            continue
        m = _AES.match(ln)
        if m:
            cur = None
            recs.append({"cipher": "AES", "label": m[1], "bytes": int(m[2]), "threads": int(m[3]),
                         "keygen_us": None, "us": _nums(m[4])})
            continue
        m = _GPU.match(ln)
        if m:
            cur = None
            recs.append({"cipher": "AES", "label": "AES ECB test", "bytes": int(m[1]), "threads": 1,
                         "keygen_us": None, "us": _nums(m[2]), "average_us": int(m[3])})
            continue
        if cur is not None and re.fullmatch(r"[\d, ]+", ln or "x"):
            cur["us"].extend(_nums(ln))
    return recs


def summarize(rec: dict) -> dict:
    """Median of iterations 2..N (the first is a cold outlier) and best, in
    GB/s (decimal) -- the convention of BASELINE.md."""
    us = rec["us"][1:] if len(rec["us"]) > 1 else rec["us"]
    med = statistics.median(us) if us else float("nan")
    best = min(us) if us else float("nan")
    return {**rec, "median_us": med, "gbps_median": rec["bytes"] / med / 1e3 if med else None,
            "gbps_best": rec["bytes"] / best / 1e3 if best else None}


class JsonlWriter:
    def __init__(self, path: str):
        self.path = path

    def write(self, **rec):
        with open(self.path, "a") as f:
            f.write(json.dumps(rec, sort_keys=True) + "\n")


def split_sections(text: str) -> list[list[dict]]:
    """The records of a log in the order printed, cut at lines that are not
    records: the ARC4 self-test lines end the CPU sweep of bin/test (so a
    bin/test log followed by a ``--device gpu`` log gives two sections) and
    ``## `` lines head a bin/aes_test log."""
    chunks, cur = [], []
    for ln in text.splitlines():
        if ln.strip().startswith("ARC4 test #") or ln.startswith("## "):
            chunks.append(cur)
            cur = []
        else:
            cur.append(ln)
    chunks.append(cur)
    return [recs for recs in (parse("\n".join(c) + "\n") for c in chunks) if recs]


def gbps_table(records: list[dict]) -> dict:
    """(label, bytes, threads) -> median-of-iterations-2..N GB/s (summarize)."""
    return {(r["label"], r["bytes"], r["threads"]): summarize(r)["gbps_median"] for r in records}
