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
