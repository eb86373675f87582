"""The work-claiming protocol of the co-resident split (csrc/hip/otc_device.h
claim_unit, engine.cpp split_claim), replayed on the host: any interleaving
of front (bitsliced, a whole task of TASK units) and back (T-table, one unit)
claims on the one 64-bit counter hands out every unit exactly once, with the
bitsliced tasks aligned and clear of the reserve, including the claims that
arrive after the buffer is exhausted (they still add to the counter)."""
import random

import pytest


TASKS = (1, 2)  # units per bitsliced task, 2048 / OTC_CLAIM_UNIT: shipped 1, the A/B build 2


def claim(counter, nunits, back, reserve=0, TASK=1):
    """the soft reserve check (a plain read, no add), then one atomic add on
    the word + the validity rule; returns (counter, claimed units)"""
    f, b = counter & 0xFFFFFFFF, counter >> 32
    if not back and reserve and f + b + TASK + reserve > nunits:
        return counter, None  # stop without adding
    old = counter
    counter = (counter + ((1 << 32) if back else TASK)) & ((1 << 64) - 1)
    f, b = old & 0xFFFFFFFF, old >> 32
    if f + b >= nunits:
        return counter, None
    if back:
        return counter, [nunits - 1 - b]
    assert f % TASK == 0
    half = f + b + TASK > nunits  # CLAIM_HALF: only the task's first unit
    return counter, [f] if half else list(range(f, f + TASK))


@pytest.mark.parametrize("task", TASKS)
@pytest.mark.parametrize("seed", range(60))
def test_every_unit_once(seed, task):
    rnd = random.Random(seed)
    nunits = rnd.choice([1, 4, 5, 7, 64, 1000, 4097])
    reserve = rnd.choice([0, 0, 1, 3, 100])
    front_waves, back_waves = rnd.randint(1, 40), rnd.randint(1, 200)
    waves = [("f", i) for i in range(front_waves)] + [("b", i) for i in range(back_waves)]
    live = set(waves)
    counter, got = 0, []
    while live:
        w = rnd.choice(sorted(live))  # any wave may claim next: the atomics' order
        counter, us = claim(counter, nunits, w[0] == "b", reserve, task)
        if us is None:
            live.discard(w)  # a wave stops at its first failed claim
        else:
            got += [(u, w[0]) for u in us]
    units = sorted(u for u, _ in got)
    assert units == list(range(nunits))  # all, none twice
    # the bitsliced side holds a prefix, the T-table side the matching suffix
    front = sorted(u for u, s in got if s == "f")
    assert front == list(range(len(front)))


@pytest.mark.parametrize("task", TASKS)
def test_reserve_is_soft_but_kept_without_races(task):
    """With claims in sequence (no read-to-add race), the bitsliced side
    stops with more than `reserve` units left to the T-table."""
    nunits, reserve = 1000, 37
    counter, front = 0, 0
    while True:
        counter, us = claim(counter, nunits, False, reserve, task)
        if us is None:
            break
        front += len(us)
    assert nunits - front >= reserve and front % task == 0


def test_counter_halves_cannot_carry():
    """Counts stay far below 2^32 (units <= 2^31 - 1, plus one failed claim
    per wave), so the front half never carries into the back half."""
    nunits = (1 << 31) - 1
    waves = 1 << 14
    assert nunits + waves < (1 << 32)
