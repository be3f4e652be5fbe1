"""renderer.acquire_stream / release_stream (host logic, CPU): a live renderer's streams are distinct, a closed
renderer's streams go back to the bucket (device, priority) they came from and the next renderer reuses them, so a
run of many renderers does not walk through torch's fixed per-priority pool (whose 33rd stream would alias the
1st, and possibly a process group's communication stream). torch.cuda is stood in for; the GPU test
test_gpu_parity.py::test_renderer_streams_distinct_and_recycled checks the real streams."""
import itertools

import pytest


class _FakeStream:
    _ids = itertools.count()

    def __init__(self, priority=0):
        self.priority = max(priority, -1)  # a clamped priority, as torch may report
        self.id = next(self._ids)


@pytest.fixture
def pool(monkeypatch):
    import torch

    from ptsvgf import renderer as R

    monkeypatch.setattr(torch.cuda, "Stream", _FakeStream)
    monkeypatch.setattr(torch.cuda, "current_device", lambda: 0)
    monkeypatch.setattr(R, "_FREE_STREAMS", {})
    return R


def test_streams_distinct_then_recycled(pool):
    a = [pool.acquire_stream() for _ in range(4)] + [pool.acquire_stream(-1)]
    assert len({s.id for s in a}) == 5
    for s in a:
        pool.release_stream(s)
    b = [pool.acquire_stream() for _ in range(4)] + [pool.acquire_stream(-1)]
    assert {s.id for s in b} == {s.id for s in a}          # reused, no new allocations
    assert b[-1].id == a[-1].id                             # the high-priority one back from its own bucket


def test_clamped_priority_returns_to_its_bucket(pool):
    s = pool.acquire_stream(-3)  # torch reports -1 for it; the pool keys by what was asked
    pool.release_stream(s)
    assert pool.acquire_stream(-3) is s
    assert pool.acquire_stream(-1) is not s


def test_release_ignores_foreign_and_none(pool):
    pool.release_stream(None)
    pool.release_stream(_FakeStream())  # not from the pool: not adopted
    assert all(not v for v in pool._FREE_STREAMS.values())
