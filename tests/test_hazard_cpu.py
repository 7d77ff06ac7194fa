"""The side/main graph hazard checker's analysis (rocfm/utils/hazard.py) on synthetic launches.

The GPU suite runs every engine with ROCFM_HAZARD=1 (tests/test_hazard_gpu.py); these tests pin the
checker itself: role parsing from the bindings, pointer discovery in parameter blocks (named
fields and raw bytes), per-parity extents, and that a shared written buffer is reported."""
import struct

import pytest

from rocfm.utils import hazard as Z


def test_pointer_roles_from_bindings():
    roles = Z.pointer_roles()
    assert roles["RowsParams"]["ids"] is False  # const int32_t*
    assert roles["RowsParams"]["contrib"] is True  # float*
    assert roles["SortAuxParams"]["pos"] is True
    assert "cls" not in roles


class _Map(Z.TensorMap):
    def __init__(self, items):
        super().__init__()
        self._items = list(items)


class SortAuxParams:  # named like the binding so its ROCFM_PTR roles apply
    def __init__(self, **kw):
        for f in Z.pointer_roles()["SortAuxParams"]:
            setattr(self, f, 0)
        self.__dict__.update(kw)
        self.extra = []

    def raw(self):
        vals = [getattr(self, f) for f in sorted(Z.pointer_roles()["SortAuxParams"])] + self.extra
        return b"".join(struct.pack("<Q", v) for v in vals) + b"\x00" * 4


class RowsParams(SortAuxParams):
    def __init__(self, **kw):
        for f in Z.pointer_roles()["RowsParams"]:
            setattr(self, f, 0)
        self.__dict__.update(kw)
        self.extra = []

    def raw(self):
        vals = [getattr(self, f) for f in sorted(Z.pointer_roles()["RowsParams"])] + self.extra
        return b"".join(struct.pack("<Q", v) for v in vals)


BASE = 0x7F0000000000
TMAP = _Map([(BASE, BASE + 4096, "eng.m_pos"),           # one allocation, two parity halves
             (BASE + 8192, BASE + 12288, "eng.emb"),
             (BASE + 16384, BASE + 20480, "eng.weights")])


def _rec(side_calls, main_calls):
    r = Z.Recorder()
    r.begin("side")
    for name, args in side_calls:
        r.note(name, args)
    r.begin("main")
    for name, args in main_calls:
        r.note(name, args)
    r.end()
    return r


def test_parity_halves_do_not_conflict():
    side = [("sort_aux", (SortAuxParams(pos=BASE + 2048),))]          # writes parity 1's half
    main = [("deepfm_rows", (RowsParams(contrib_pos=BASE, emb=BASE + 8192),))]  # reads parity 0's half
    r = _rec(side, main)
    xs, ys = r.accesses("side", TMAP), r.accesses("main", TMAP)
    assert [a.field for a in xs] == ["pos"] and xs[0].write
    assert {a.field for a in ys} == {"contrib_pos", "emb"} and not any(a.write for a in ys)
    assert Z.conflicts(xs, ys) == []


def test_shared_written_buffer_is_reported():
    side = [("sort_aux", (SortAuxParams(pos=BASE),))]
    main = [("deepfm_rows", (RowsParams(contrib_pos=BASE),))]
    r = _rec(side, main)
    found = Z.conflicts(r.accesses("side", TMAP), r.accesses("main", TMAP))
    assert len(found) == 1 and found[0][0].field == "pos" and found[0][1].field == "contrib_pos"


def test_reads_only_and_raw_pointers():
    # both read the table: no hazard; a pointer set through a set_* array (raw bytes only) counts as a write
    p = RowsParams(emb=BASE + 8192)
    p.extra = [BASE + 16384 + 64]
    r = _rec([("x", (RowsParams(emb=BASE + 8192),))], [("deepfm_rows", (p,))])
    xs, ys = r.accesses("side", TMAP), r.accesses("main", TMAP)
    assert Z.conflicts(xs, ys) == []
    assert any(a.owner == "eng.weights" and a.write and a.field.startswith("@") for a in ys)
    # a plain integer argument into a known buffer (sort launchers) is a write
    r2 = _rec([("sort_pairs", (BASE + 16384 + 64, 123))], [("deepfm_rows", (p,))])
    found = Z.conflicts(r2.accesses("side", TMAP), r2.accesses("main", TMAP))
    assert len(found) == 1 and found[0][0].field == "arg0"


def test_check_raises_with_report(monkeypatch):
    r = _rec([("sort_aux", (SortAuxParams(pos=BASE),))], [("deepfm_rows", (RowsParams(contrib_pos=BASE),))])
    monkeypatch.setattr(Z.TensorMap, "from_roots", classmethod(lambda cls, roots: TMAP))
    with pytest.raises(Z.HazardError, match=r"sort_aux\.pos W eng\.m_pos\+0.*deepfm_rows\.contrib_pos R"):
        r.check("test")


def test_proxy_notes_calls_and_passes_classes():
    class Mod:
        class RowsParams:
            pass

        @staticmethod
        def launch(a, b):
            return a + b

    r = Z.Recorder()
    px = Z.HipProxy(Mod, r)
    assert px.RowsParams is Mod.RowsParams
    r.begin("main")
    assert px.launch(1, 2) == 3
    assert r.calls["main"] == [("launch", (1, 2))]


# ---- the streamed loop's three-stream plan (StreamPlan) ------------------------------------------
def test_stream_plan_orders_through_waits_transitively():
    from rocfm.utils.hazard import HazardError, StreamPlan

    p = StreamPlan()
    p.op("copy", "fill slot 0", [("ring", 0, 1, True)])
    t = p.record("copy")
    p.op("side", "unrelated")
    p.wait("side", t)
    p.op("side", "read slot 0", [("ring", 0, 1, False)])
    t2 = p.record("side")
    p.wait("main", t2)
    p.op("main", "m")
    p.wait("copy", p.record("main"))
    p.op("copy", "refill slot 0", [("ring", 0, 1, True)])  # ordered after the read via main
    assert p.conflicts() == []
    p.check()
    q = StreamPlan()
    q.op("copy", "fill", [("ring", 2, 4, True)])
    q.op("side", "read", [("ring", 3, 5, False)])  # no wait: unordered overlap
    q.op("main", "read elsewhere", [("ring", 4, 5, False)])
    found = q.conflicts()
    assert found == [("ring", "copy:fill", "side:read")]
    with pytest.raises(HazardError, match="copy:fill"):
        q.check("t")


def _simulate_train_stream(S: int, graphs: int, early: bool, skip_init_wait: bool = False, early_at: int = 3,
                           check_every: bool = False):
    """The event plan of FusedDeepFM.train_stream / _launch_multi on a 4·S-slot ring, in plan ops
    (``early``: from graph ``early_at`` on, the refill waits one side graph too early;
    ``check_every``: check — and so prune — after every graph, as the loop does)."""
    from rocfm.utils.hazard import StreamPlan

    R = 4 * S
    p = StreamPlan()
    staged = 0

    def stage(k):
        nonlocal staged
        p.op("copy", f"stage {staged}", [("ring", staged % R, staged % R + k, True)])
        staged += k
        return p.record("copy")

    p.op("main", "ring allocation (zero fill)", [("ring", 0, R, True)])
    if not skip_init_wait:
        p.wait_stream("copy", "main")
    cevs = [stage(2 * S)]
    p.wait("main", cevs[0])
    p.op("main", "prime", [("ring", 0, S, False), ("m_batches", 0, 1, True)])
    prime = p.record("main")
    sevs, side_ev, i = [], None, 0
    for j in range(graphs):
        w = sevs[j - 3] if j >= 3 else prime
        if early and j >= max(3, early_at):
            w = sevs[j - 4] if j >= 4 else prime
        p.wait("copy", w)
        cevs.append(stage(S))
        p.wait("side", cevs[j])
        q = j % 2
        before = p.record("main")
        p.wait("main", side_ev)
        p.op("main", f"main {j}", [("m_batches", q, q + 1, False)])
        p.wait("side", before)
        lo = (i + S) % R
        p.op("side", f"side {j}", [("ring", lo, lo + S, False), ("m_batches", 1 - q, 2 - q, True)])
        side_ev = p.record("side")
        sevs.append(side_ev)
        i += S
        if check_every:
            p.check(f"graph {j}")
    return p


def test_train_stream_event_plan_is_race_free_and_an_early_refill_is_caught():
    """The loop's plan (copy refills wait for the side graph three back) has no unordered access;
    waiting one side graph too early lets a refill overwrite ring slots a side graph may still be
    reading — the checker names both operations."""
    from rocfm.utils.hazard import HazardError

    for S in (2, 4, 16):
        _simulate_train_stream(S, 12, early=False).check()
    bad = _simulate_train_stream(4, 12, early=True)
    found = bad.conflicts()
    assert found and all(n == "ring" for n, _, _ in found)
    assert any(a.startswith("copy:stage") and b.startswith("side:side") or
               b.startswith("copy:stage") and a.startswith("side:side") for _, a, b in found)
    with pytest.raises(HazardError):
        bad.check()
    # the first refill racing the ring's zero fill on the compute stream (no copy.wait_stream(main))
    found = _simulate_train_stream(4, 3, early=False, skip_init_wait=True).conflicts()
    assert any("ring allocation" in a or "ring allocation" in b for _, a, b in found)


def test_stream_plan_stays_bounded_over_an_epoch_and_still_catches_a_late_race():
    """Checked after every graph (as train_stream does), the plan prunes itself to its window: a
    5,000-graph stream keeps ≤ window operations, and an early refill injected at graph 4,000 is
    still caught."""
    from rocfm.utils.hazard import HazardError

    p = _simulate_train_stream(8, 5000, early=False, check_every=True)
    assert len(p.ops) <= p.window and p.base > 14000
    with pytest.raises(HazardError, match="copy:stage"):
        _simulate_train_stream(8, 4100, early=True, early_at=4000, check_every=True)


def test_observed_write_catches_unannotated_copy():
    """An un-annotated copy into the ring (no ``plan.op`` for it) is still seen: ObservedWrites turns
    the aten write into a plan operation on the issuing stream, so a refill that races a side-chain
    read raises, and the same refill behind the side stream's event does not."""
    import torch
    from rocfm.utils.hazard import HazardError, ObservedWrites, StreamPlan

    ring = torch.zeros(8, 4, 3)
    src = torch.ones(2, 4, 3)
    for ordered in (False, True):
        plan = StreamPlan()
        cur = ["side"]
        plan.op("side", "side graph reads slots 2..5", [("ring", 2, 6, False)])
        if ordered:
            plan.wait_stream("copy", "side")
        cur[0] = "copy"
        with ObservedWrites(plan, {"ring": [ring]}, stream_of=lambda: cur[0]) as obs:
            ring[3:5].copy_(src)  # the undeclared refill
            torch.zeros(3).add_(1.0)  # a write outside the ring: not an operation
        assert obs.seen == 1
        assert plan.ops[-1][2] == [("ring", 3, 5, True)]
        if ordered:
            plan.check()
        else:
            with pytest.raises(HazardError, match="observed"):
                plan.check()
