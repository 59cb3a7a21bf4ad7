"""parallel.SlotRing: with `slots` buffer sets and a main-stream wait only
every `wait_every` submits, every submit may reuse its set only after the
side work of the submit `slots` back is done (side work completes in order,
so one wait covers everything up to the event it names)."""
import pytest

from prysm_amd.parallel import SlotRing


class _Stream:
    def __init__(self):
        self.done_upto = -1  # the main stream has waited for side work <= this submit
        self.waits = 0

    def wait_event(self, ev):
        self.done_upto = max(self.done_upto, ev)
        self.waits += 1


@pytest.mark.parametrize("slots,every", [(2, 1), (3, 1), (3, 2), (4, 2), (4, 3), (6, 3)])
def test_reuse_only_after_side_work_done(slots, every):
    ring, cur = SlotRing(slots, every), _Stream()
    for m in range(60):
        s = ring.acquire(cur)
        assert s == m % slots
        # set s was last used by submit m - slots: its side work must be covered
        assert m - slots < 0 or cur.done_upto >= m - slots, (m, cur.done_upto)
        ring.release(m)  # the "event" is the submit index
    assert cur.waits <= -(-60 // every)
    assert len(ring._ev) <= slots


def test_cpu_mode_and_bad_args():
    ring = SlotRing(3, 1)
    got = []
    for _ in range(5):
        got.append(ring.acquire(None))
        ring.release(None)
    assert got == [0, 1, 2, 0, 1]
    with pytest.raises(ValueError):
        SlotRing(2, 2)
    with pytest.raises(ValueError):
        SlotRing(3, 0)
