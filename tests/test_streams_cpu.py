"""ops/streams.py on the CPU: weight-gradient work runs in order (there is no side stream), the
joins and the collective context are no-ops, and the auto mode's token threshold."""
import contextlib

import torch

from mingpt_distributed_amd.ops import streams


def test_cpu_weight_gradient_runs_in_order():
    out = torch.zeros(4)
    x = torch.ones(4)
    streams.run_wgrad(lambda: out.add_(x), x)
    assert torch.equal(out, torch.ones(4))  # done before run_wgrad returned
    assert not streams.pending()
    streams.join()  # nothing in flight: a no-op
    with streams.collective_stream(torch.device("cpu")):
        out.add_(1)
    assert torch.equal(out, torch.full((4,), 2.0))


def test_auto_threshold_and_switches():
    prev = (streams._ENABLED, streams._MODE)
    try:
        streams.set_enabled(True, "auto")
        assert streams.use_for(streams._AUTO_TOKENS)
        assert not streams.use_for(streams._AUTO_TOKENS + 1)
        streams.set_enabled(True, "1")
        assert streams.use_for(10 ** 6)
        streams.set_enabled(False)
        assert not streams.use_for(1)
    finally:
        streams._ENABLED, streams._MODE = prev


def test_ddp_launch_uses_collective_context(monkeypatch):
    """The data-parallel engine issues a bucket's collective inside streams.collective_stream (so
    on GPUs it is ordered after the side-stream weight gradients of that bucket)."""
    from mingpt_distributed_amd.parallel import ddp

    entered = []

    @contextlib.contextmanager
    def spy(device):
        entered.append(device)
        yield

    monkeypatch.setattr(ddp.streams, "collective_stream", spy)

    class _B:
        start, end, params, work = 0, 4, [], None

    class _Eng(ddp.DataParallelEngine):
        def __init__(self):  # only what _launch touches
            self.next_launch = 0
            self.inflight = []
            self.store = type("S", (), {"device": torch.device("cpu")})()

        def _issue(self, b, wire=None):
            return "work"

    e = _Eng()
    b = _B()
    e._launch(b)
    assert entered == [torch.device("cpu")] and b.work == "work"


def test_compute_priority_modes(monkeypatch):
    """MINGPT_COMPUTE_PRIORITY: "auto" raises the compute stream's priority exactly where the
    side stream runs the weight gradients; "off" never; an integer always; CPU: no stream."""
    prev = (streams._ENABLED, streams._MODE)
    try:
        streams.set_enabled(True, "auto")
        monkeypatch.setattr(streams, "_COMPUTE_PRIO", "auto")
        assert streams.compute_priority(16384) == -1
        assert streams.compute_priority(16384, 1600) == -1  # gpt2-xl at B = 16
        assert streams.compute_priority(8192, 192) is None  # gpt-mini: launch-bound, no side stream
        assert not streams.use_for(8192, 192) and streams.use_for(8192, 768)
        assert streams.compute_priority(131072) is None
        monkeypatch.setattr(streams, "_COMPUTE_PRIO", "off")
        assert streams.compute_priority(16384) is None
        monkeypatch.setattr(streams, "_COMPUTE_PRIO", "-1")
        assert streams.compute_priority(131072) == -1
        with streams.compute_stream(torch.device("cpu"), 16):
            pass  # a no-op on the CPU
    finally:
        streams._ENABLED, streams._MODE = prev
