"""The work-claiming protocol of the co-resident split (csrc/hip/otc_device.h
claim_unit, engine.cpp split_claim), replayed on the host: any interleaving
of front (bitsliced) and back (T-table) claims on the one 64-bit counter hands
out every unit exactly once, including the claims that arrive after the
buffer is exhausted (they still add to the counter)."""
import random

import pytest


def claim(counter, nunits, back):
    """one atomic add on the word + the validity rule; returns (counter, unit or -1)"""
    old = counter
    counter = (counter + ((1 << 32) if back else 1)) & ((1 << 64) - 1)
    f, b = old & 0xFFFFFFFF, old >> 32
    if f + b >= nunits:
        return counter, -1
    return counter, (nunits - 1 - b) if back else f


@pytest.mark.parametrize("seed", range(40))
def test_every_unit_once(seed):
    rnd = random.Random(seed)
    nunits = rnd.choice([1, 2, 3, 7, 64, 1000, 4097])
    front_waves, back_waves = rnd.randint(1, 40), rnd.randint(1, 200)
    waves = [("f", i) for i in range(front_waves)] + [("b", i) for i in range(back_waves)]
    live = set(waves)
    counter, got = 0, []
    while live:
        w = rnd.choice(sorted(live))  # any wave may claim next: the atomics' order
        counter, u = claim(counter, nunits, w[0] == "b")
        if u < 0:
            live.discard(w)  # a wave stops at its first failed claim
        else:
            got.append((u, w[0]))
    units = sorted(u for u, _ in got)
    assert units == list(range(nunits))  # all, none twice
    # the bitsliced side holds a prefix, the T-table side the matching suffix
    front = sorted(u for u, s in got if s == "f")
    assert front == list(range(len(front)))


def test_counter_halves_cannot_carry():
    """Counts stay far below 2^32 (units <= 2^31 - 1, plus one failed claim
    per wave), so the front half never carries into the back half."""
    nunits = (1 << 31) - 1
    waves = 1 << 14
    assert nunits + waves < (1 << 32)
