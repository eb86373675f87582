"""The generated S-box header is pinned to its generator's recorded output
(tools/sbox77_cover.json, written from tools/sbox_choices.py + sbox_schedule.py):
the recorded program computes S(x ^ k) for all 2^16 (x, k) with the recorded
peak of live planes, and the shipped header body is exactly what
tools/sbox_cover.py emits from it -- a hand edit of the header, or of the
record, fails (round-3 review, next-round item 7)."""
import json
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TOOL = os.path.join(ROOT, "tools", "sbox_cover.py")
COVER = os.path.join(ROOT, "tools", "sbox77_cover.json")
HDR = os.path.join(ROOT, "csrc", "include", "otc_sbox_lut3.h")


def check(cover=COVER, hdr=HDR):
    return subprocess.run([sys.executable, TOOL, "emit", cover, hdr, "--check"], capture_output=True, text=True,
                          timeout=120)


def test_shipped_header_matches_generator_record():
    r = check()
    assert r.returncode == 0, r.stderr
    c = json.load(open(COVER))
    assert c["luts"] == 77 and c["peak_live"] == 23 and len(c["statements"]) == 77


def test_hand_edited_header_fails(tmp_path):
    text = open(HDR).read()
    # (a) one LUT immediate changed
    m = re.search(r"(lut3\(\w+, \w+, \w+, 0x)([0-9a-f]{2})\)", text)
    bad = text[:m.start(2)] + "%02x" % (int(m.group(2), 16) ^ 0x01) + text[m.end(2):]
    p = tmp_path / "a.h"
    p.write_text(bad)
    r = check(hdr=str(p))
    assert r.returncode == 1 and "generator emits" in r.stderr
    # (b) two statements swapped (same function, different schedule)
    lines = text.split("\n")
    i = next(k for k, ln in enumerate(lines) if ln.startswith("    W T7 ="))
    lines[i], lines[i + 1] = lines[i + 1], lines[i]
    p = tmp_path / "b.h"
    p.write_text("\n".join(lines))
    assert check(hdr=str(p)).returncode == 1


def test_corrupted_record_fails(tmp_path):
    c = json.load(open(COVER))
    n, e = c["statements"][-1]
    c["statements"][-1] = [n, e.replace("0x69", "0x96") if "0x69" in e else e.replace("0x96", "0x69")]
    p = tmp_path / "c.json"
    p.write_text(json.dumps(c))
    r = check(cover=str(p))
    assert r.returncode == 1 and "is not bit" in r.stderr
