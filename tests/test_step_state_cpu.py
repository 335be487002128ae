"""The step-state ring's host-side bookkeeping (qat.StepState.stage / launched) without a GPU: a
slot is rewritten only after an event recorded after the replay that last read it, and the host is
never held back more than the event spacing requires.  The events are stand-ins that remember the
replay count they were recorded at; the ring's device fetch is covered by test_step_state_gpu."""
import numpy as np
import pytest
import torch


class _Event:
    log = []
    current = 0

    def __init__(self):
        self.count = None

    def record(self):
        self.count = _Event.current

    def synchronize(self):
        _Event.log.append(self.count)


@pytest.mark.parametrize("ring", [32, 64, 128])
def test_ring_slot_waits_cover_the_last_reader(monkeypatch, ring):
    from quantizationawarethzdoe_amd import qat
    monkeypatch.setattr(torch.Tensor, "pin_memory", lambda self: self)
    monkeypatch.setattr(torch.cuda, "Event", _Event)
    ss = qat.StepState(torch.device("cpu"), seed=3, device_rng=True, nz=1, ring=ring)
    ev = ss.EVERY
    for f in range(5 * ring):
        _Event.log = []
        ss.stage([0.5, 1.0, 0.25], f, [0.01 * f])
        if f < ring:
            assert _Event.log == []  # a slot's first use: nothing to wait for
        else:
            assert len(_Event.log) == 1
            c = _Event.log[0]
            # the replay that last read slot f % ring is replay f - ring, counted f - ring + 1
            assert c is not None and c >= f - ring + 1
            assert c <= f - ring + ev  # the earliest such event: the host may run ring - EVERY ahead
        row = ss._ring_host[f % ring]
        assert row[4] == f and np.float32(row[5:6].view(np.float32)[0]) == np.float32(0.01 * f)
        _Event.current = f + 1  # launched() runs after replay f: count f + 1
        ss.launched()
    assert ss._fetches == 5 * ring


def test_fill_layout():
    from quantizationawarethzdoe_amd import qat
    ss = qat.StepState.__new__(qat.StepState)
    ss._np, ss.seed = np, 77
    row = np.zeros(7, dtype=np.int32)
    ss._fill(row, [1.5, -2.0, 0.125], 2 ** 31 + 5, [0.1, 0.2])
    assert list(row[:3].view(np.float32)) == [1.5, -2.0, 0.125]
    assert row[3] == 77 and row[4] == 5  # the step wraps into a non-negative int32
    assert list(row[5:].view(np.float32)) == [np.float32(0.1), np.float32(0.2)]
