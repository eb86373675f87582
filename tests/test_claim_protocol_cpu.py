"""The co-resident split's work-claim protocol (csrc/hip/otc_device.h
claim_unit / claim_front), modelled on the CPU: one 64-bit word, front
(bitsliced) count in the low half, back (T-table) count in the high half,
every claim one atomic add.  Any interleaving of claims must hand out every
unit exactly once -- front and back claims of one unit each -- and a failed
claim takes nothing."""
import random

import pytest


def claim(counter, nunits, back):
    """one atomic add; returns (new counter, list of units claimed)"""
    f, b = counter & 0xFFFFFFFF, counter >> 32
    counter += (1 << 32) if back else 1
    if f + b >= nunits:
        return counter, []
    return counter, [nunits - 1 - b] if back else [f]


@pytest.mark.parametrize("seed", [1235, 1242])
def test_every_unit_exactly_once(seed):
    rnd = random.Random(seed)
    for _ in range(300):
        nunits = rnd.randint(1, 300)
        counter, seen, front = 0, [], []
        waves = ["b"] * rnd.randint(1, 20) + ["f"] * rnd.randint(0, 20)
        live = list(waves)
        while live:
            w = rnd.randrange(len(live))  # any wave may claim next: the atomics' order
            counter, us = claim(counter, nunits, live[w] == "b")
            if not us:
                live.pop(w)  # a wave whose claim failed exits its loop
            elif live[w] == "f":
                front += us
            seen += us
        assert sorted(seen) == list(range(nunits)), (nunits, waves)  # all, none twice
        # the bitsliced side holds a prefix, the T-table side the matching suffix
        assert sorted(front) == list(range(len(front)))


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
        counter, us = claim(counter, nunits, False)
        if not us:
            break
        seen += us
    assert seen == list(range(nunits))


def claim_pre(counter, nunits, back, pf, pb):
    """claim_unit with pre-assigned first units: the word covers the units
    between the pf first and the pb last"""
    f, b = counter & 0xFFFFFFFF, counter >> 32
    counter += (1 << 32) if back else 1
    if f + b + pf + pb >= nunits:
        return counter, []
    return counter, [nunits - pb - 1 - b] if back else [pf + f]


@pytest.mark.parametrize("seed", [21, 22])
def test_preassigned_first_units(seed):
    """engine.cpp split_claim hands the T-table waves (w < pb) unit
    nunits - 1 - w and the bitsliced waves (j < pf) unit j before any claim
    (otc_device.h first_unit): with any interleaving every unit is still
    taken exactly once, the front holds a prefix."""
    rnd = random.Random(seed)
    for _ in range(300):
        nunits = rnd.randint(1, 300)
        nb, nf = rnd.randint(1, 24), rnd.randint(0, 12)
        pb = min(nunits, nb)
        pf = min(nunits - pb, nf)
        seen = [nunits - 1 - w for w in range(pb)] + list(range(pf))
        front = list(range(pf))
        counter = 0
        live = ["b"] * nb + ["f"] * nf
        while live:
            w = rnd.randrange(len(live))
            counter, us = claim_pre(counter, nunits, live[w] == "b", pf, pb)
            if not us:
                live.pop(w)
            elif live[w] == "f":
                front += us
            seen += us
        assert sorted(seen) == list(range(nunits)), (nunits, nb, nf)
        assert sorted(front) == list(range(len(front)))
