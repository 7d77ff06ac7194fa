"""Producer-side push (csrc/kernels/push.h) plumbing that needs no GPU: the switch that decides
whether an exchange's producers push, and the kernel parameter bindings it fills."""
import types

import pytest

from rocfm.ops import hip
from rocfm.parallel.p2p import producer_push_enabled


def _ex(W, shared):
    return types.SimpleNamespace(W=W, shared_device=shared, H=hip())


@pytest.mark.parametrize("env,W,shared,want", [
    (None, 8, False, True),    # one GPU per rank on a node: on by default
    (None, 4, True, False),    # ranks sharing a GPU (rehearsal): copy push
    ("1", 4, True, True),      # forced
    ("0", 2, False, False),    # off
    ("1", 16, False, False),   # beyond one node's 8 destinations
])
def test_producer_push_switch(monkeypatch, env, W, shared, want):
    if env is None:
        monkeypatch.delenv("ROCFM_DP_PUSH", raising=False)
    else:
        monkeypatch.setenv("ROCFM_DP_PUSH", env)
    assert producer_push_enabled(_ex(W, shared)) is want


def test_producer_push_switch_rejects_unknown(monkeypatch):
    monkeypatch.setenv("ROCFM_DP_PUSH", "yes")
    with pytest.raises(ValueError):
        producer_push_enabled(_ex(2, False))


def test_push_target_bindings():
    H = hip()
    assert H.push_max_world() == 8
    t = H.PushTarget()
    assert t.W == 0  # zero-initialised: kernels take their non-push path
    t.W, t.rank, t.spin_limit = 2, 1, 1 << 20
    t.set_dest(0, 4096, 8192)
    with pytest.raises(ValueError):
        t.set_dest(8, 0, 0)
    rp, wp, ep = H.RowsParams(), H.WgradParams(), H.EmbUpdateParams()
    assert rp.push.W == 0 and rp.push2.W == 0 and wp.push.W == 0 and ep.push.W == 0
    rp.push = t
    rp.push2 = t
    wp.push = t
    ep.push, ep.push_seg, ep.push_off_keys, ep.push_off_rows = t, 128, 64, 68
    assert (rp.push.W, rp.push2.rank, wp.push.spin_limit) == (2, 1, 1 << 20)
    assert (ep.push_seg, ep.push_off_keys, ep.push_off_rows) == (128, 64, 68)
