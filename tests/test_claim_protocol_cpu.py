"""The co-resident split's work-claim protocol (csrc/hip/otc_device.h
claim_unit / claim_front), modelled on the CPU: one 64-bit word, front
(bitsliced) count in the low half, back (T-table) count in the high half,
every claim one atomic add.  Any interleaving of claims must hand out every
unit exactly once -- front claims of n units (1 for the 2048-block split, 8
for the bs8 segment-encryption kernel, which gets a partial task at the
meeting point) and back claims of one -- and a failed claim takes nothing."""
import random

import pytest


def claim(counter, nunits, back, n=1):
    """one atomic add; returns (new counter, list of units claimed)"""
    f, b = counter & 0xFFFFFFFF, counter >> 32
    counter += (1 << 32) if back else n
    used = f + b
    if used >= nunits:
        return counter, []
    if back:
        return counter, [nunits - 1 - b]
    got = min(n, nunits - used)
    return counter, list(range(f, f + got))


@pytest.mark.parametrize("n", [1, 8])
def test_every_unit_exactly_once(n):
    rnd = random.Random(1234 + n)
    for _ in range(300):
        nunits = rnd.randint(1, 300)
        counter, seen, front = 0, [], []
        waves = ["b"] * rnd.randint(1, 20) + ["f"] * rnd.randint(0, 20)
        live = list(waves)
        while live:
            w = rnd.randrange(len(live))  # any wave may claim next: the atomics' order
            counter, us = claim(counter, nunits, live[w] == "b", n)
            if not us:
                live.pop(w)  # a wave whose claim failed exits its loop
            elif live[w] == "f":
                front += us
            seen += us
        assert sorted(seen) == list(range(nunits)), (nunits, waves)  # all, none twice
        # the bitsliced side holds a prefix, the T-table side the matching suffix
        assert sorted(front) == list(range(len(front)))


def test_front_partial_task_at_the_meeting_point():
    """A bs8 front claim with fewer than 8 units left gets exactly the rest
    (its chains past the claim load chain 0 and store nothing), and later
    claims of either side fail."""
    counter = 0
    counter, us = claim(counter, 19, False, 8)
    assert us == list(range(8))
    counter, us = claim(counter, 19, True)
    assert us == [18]
    counter, us = claim(counter, 19, False, 8)
    assert us == list(range(8, 16))
    counter, us = claim(counter, 19, False, 8)
    assert us == [16, 17]
    for back in (True, False):
        counter, us = claim(counter, 19, back, 8)
        assert us == []


def test_bitsliced_only_mode():
    """impl "bitslice": the T-table kernel's own word starts at
    back = nunits, so every one of its claims fails and the front side alone
    takes every unit."""
    nunits = 37
    tt_word = nunits << 32
    tt_word, us = claim(tt_word, nunits, True)
    assert us == []
    counter, seen = 0, []
    while True:
        counter, us = claim(counter, nunits, False, 8)
        if not us:
            break
        seen += us
    assert seen == list(range(nunits))
