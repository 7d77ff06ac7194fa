"""bench.py's warm-up order (warm_capture_first): the same W untimed steps and K timed steps as the
plain order, with every graph of the last warm-up steps and of the timed window captured before
those warm-up steps run (profiles/r6_window_fixed_cost.md).  CPU: a recording stand-in engine."""
import importlib.util
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench():
    spec = importlib.util.spec_from_file_location("rocfm_bench", os.path.join(ROOT, "bench.py"))
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


class _Inner:
    def __init__(self):
        self._m_warm = 0


class _DPStandIn:
    """A DP-style engine: shadow-validated steps first, then the multi-step graphs."""

    def __init__(self, shadow_steps=0):
        self.eng = _Inner()
        self.calls = []
        self.shadow_left = shadow_steps

    @property
    def shadow(self):
        outer = self

        class S:
            @property
            def active(self):
                return outer.shadow_left > 0
        return S()

    def train_steps(self, n, spg):
        while n > 0 and self.shadow_left > 0:
            self.train_step()
            n -= 1
        if n > 0:
            self.calls.append(("steps", n))
            self.eng._m_warm += 1

    def train_step(self):
        self.shadow_left -= 1
        self.calls.append(("step", 1))

    def precapture(self, n, spg):
        self.calls.append(("capture", n))


@pytest.mark.parametrize("W", [2, 5, 8])
def test_capture_first_keeps_step_counts_and_captures_before_the_last_warmup(W, monkeypatch):
    monkeypatch.delenv("ROCFM_BENCH_CAPTURE_FIRST", raising=False)
    b = _bench()
    eng = _DPStandIn()
    assert b.warm_capture_first(eng, lambda n: eng.train_steps(n, 20), W, 20, 20)
    steps = sum(n for kind, n in eng.calls if kind in ("steps", "step"))
    assert steps == W  # exactly W untimed steps
    m = W // 2
    assert eng.calls == [("steps", W - m), ("capture", [m, 20]), ("steps", m)]


def test_capture_first_falls_back_when_only_shadow_steps_ran(monkeypatch):
    monkeypatch.delenv("ROCFM_BENCH_CAPTURE_FIRST", raising=False)
    b = _bench()
    eng = _DPStandIn(shadow_steps=10)  # every warm-up step is a shadow step: no graph launched yet
    assert b.warm_capture_first(eng, lambda n: eng.train_steps(n, 20), 5, 20, 20)
    assert eng.calls[-1] == ("capture", 20)  # the round-5 order: capture after the warm-up
    # W - m = 3 warm-up steps (shadow), the shadow drain (7), then the last m = 2 as graph steps
    assert sum(n for kind, n in eng.calls if kind == "step") == 10
    assert eng.calls[-2] == ("steps", 2)


def test_capture_first_off(monkeypatch):
    b = _bench()
    eng = _DPStandIn()
    monkeypatch.setenv("ROCFM_BENCH_CAPTURE_FIRST", "0")
    assert not b.warm_capture_first(eng, lambda n: eng.train_steps(n, 20), 5, 20, 20)
    monkeypatch.delenv("ROCFM_BENCH_CAPTURE_FIRST")
    assert not b.warm_capture_first(eng, lambda n: eng.train_steps(n, 20), 1, 20, 20)  # W < 2
    assert eng.calls == []
