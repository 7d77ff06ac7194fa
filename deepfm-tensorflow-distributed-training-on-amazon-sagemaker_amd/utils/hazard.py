"""Cross-stream hazard checker for the two-graph multi-step launches (``ROCFM_HAZARD=1``).

Every multi-step launch is a side graph (the next group's fetch, sort, sort aux, dedup; the
row-shard routing) on the sort stream, running concurrently with the main graph (the steps and,
distributed, the exchanges and merges) on the compute stream (``FusedDeepFM._launch_multi``).  The
two share no buffer by construction: the side graph fills the parity 1-q buffers while the main
graph consumes parity q.  Nothing enforces that, however — a buffer added to both chains without a
parity index is a race that shows up only as rare run-to-run differences.

With ``ROCFM_HAZARD=1`` the engine's extension handle is wrapped: every launcher call records the
device buffers its arguments point into, with their role, and each newly captured graph pair is
checked before it ever runs:

* a parameter block's pointer fields are read by name, with the role from the field's declared type
  in ``csrc/bindings.inc`` (``ROCFM_PTR(cls, field, const T*)`` = read, a non-const pointer = write);
* the block's raw bytes (``.raw()``) are scanned for further pointers — arrays set through the
  ``set_*`` methods (layer weights, activations, peer slots) — which count as writes (unknown role);
* plain integer arguments that point into a known buffer (the sort launchers) count as writes.

Pointers are resolved against every CUDA tensor reachable from the registered roots (the engine, and
the DP / row-shard driver): attributes, and lists / tuples / dicts of tensors.  An access covers its
tensor from its base pointer up to the next base pointer any recorded access uses inside the same
tensor (so per-parity slices of one allocation stay apart).  Two accesses, one from each graph, that
overlap with at least one write are a hazard: ``HazardError`` names both launches, fields and the
buffer.  Torch ops and collectives inside a capture are not recorded (the HIP-extension launches only).
"""
from __future__ import annotations

import bisect
import os
import re
from collections import defaultdict
from typing import Dict, List, Optional, Tuple

import torch

_ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
_BINDINGS = os.path.join(_ROOT, "csrc", "bindings.inc")
_PTR_RE = re.compile(r"ROCFM_PTR\(\s*(\w+)\s*,\s*(\w+)\s*,\s*([^)]*)\)")


class HazardError(RuntimeError):
    pass


def enabled() -> bool:
    return os.environ.get("ROCFM_HAZARD", "0") == "1"


_roles_cache: Optional[Dict[str, Dict[str, bool]]] = None


def pointer_roles(path: str = _BINDINGS) -> Dict[str, Dict[str, bool]]:
    """class name → {pointer field → writable} from the ROCFM_PTR declarations."""
    global _roles_cache
    if _roles_cache is not None and path == _BINDINGS:
        return _roles_cache
    roles: Dict[str, Dict[str, bool]] = defaultdict(dict)
    with open(path) as f:
        text = f.read()
    for cls, field, typ in _PTR_RE.findall(text):
        if cls == "cls":  # the macro's own definition
            continue
        roles[cls][field] = not typ.strip().startswith("const")
    out = dict(roles)
    if path == _BINDINGS:
        _roles_cache = out
    return out


class Access:
    __slots__ = ("section", "kernel", "field", "owner", "base", "write")

    def __init__(self, section, kernel, field, owner, base, write):
        self.section, self.kernel, self.field, self.owner, self.base, self.write = (
            section, kernel, field, owner, base, write)

    def __repr__(self):
        return f"{self.kernel}.{self.field} {'W' if self.write else 'R'} {self.owner}+{self.base}"


class TensorMap:
    """Address → the registered tensor storage holding it.  Accesses are grouped by the OUTERMOST
    registered range (the allocation) so that views kept as attributes compare with their base."""

    def __init__(self):
        self._items: List[Tuple[int, int, str]] = []

    def add(self, name: str, t: torch.Tensor) -> None:
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda" or t.numel() == 0:
            return
        lo = t.data_ptr()
        self._items.append((lo, lo + t.numel() * t.element_size(), name))

    def lookup(self, ptr: int) -> Optional[Tuple[int, int, str]]:
        """(allocation start, allocation end, name) of the outermost registered range with ptr."""
        best = None
        for lo, hi, name in self._items:
            if lo <= ptr < hi and (best is None or hi - lo > best[1] - best[0]):
                best = (lo, hi, name)
        return best

    @classmethod
    def from_roots(cls, roots) -> "TensorMap":
        m = cls()
        for prefix, obj in roots:
            for k, v in vars(obj).items():
                _add_obj(m, f"{prefix}.{k}", v, 2)
        return m


def _add_obj(m: TensorMap, name: str, v, depth: int) -> None:
    if isinstance(v, torch.Tensor):
        m.add(name, v)
    elif depth > 0 and isinstance(v, (list, tuple)):
        for i, x in enumerate(v):
            _add_obj(m, f"{name}[{i}]", x, depth - 1)
    elif depth > 0 and isinstance(v, dict):
        for k, x in v.items():
            _add_obj(m, f"{name}[{k!r}]", x, depth - 1)


class Recorder:
    """Collects the launches of the current section ("side" / "main") per graph pair."""

    def __init__(self):
        self.roots: List[Tuple[str, object]] = []
        self.section: Optional[str] = None
        self.calls: Dict[str, List[Tuple[str, tuple]]] = defaultdict(list)
        self.checked = 0

    def attach(self, prefix: str, obj) -> None:
        self.roots.append((prefix, obj))

    def begin(self, section: str) -> None:
        self.section = section
        self.calls[section] = []

    def end(self) -> None:
        self.section = None

    def note(self, name: str, args: tuple) -> None:
        if self.section is not None:
            self.calls[self.section].append((name, args))

    # ---- analysis -------------------------------------------------------------------------------
    def accesses(self, section: str, tmap: TensorMap) -> List[Access]:
        roles = pointer_roles()
        out = []
        for kernel, args in self.calls.get(section, []):
            flat = []
            for a in args:  # (a list argument: one launch over several parameter blocks)
                flat.extend(a if isinstance(a, (list, tuple)) else [a])
            for ai, a in enumerate(flat):
                if hasattr(a, "raw"):
                    named = roles.get(type(a).__name__, {})
                    seen = set()
                    for field, w in named.items():
                        v = int(getattr(a, field))
                        if v:
                            seen.add(v)
                            hit = tmap.lookup(v)
                            if hit:
                                out.append(Access(section, kernel, field, hit[2], v - hit[0], w))
                    raw = a.raw()
                    for off in range(0, len(raw) - 7, 8):
                        v = int.from_bytes(raw[off:off + 8], "little")
                        if v and v not in seen:
                            hit = tmap.lookup(v)
                            if hit:
                                seen.add(v)
                                out.append(Access(section, kernel, f"@{off}", hit[2], v - hit[0], True))
                elif isinstance(a, int) and not isinstance(a, bool) and a > 65536:
                    hit = tmap.lookup(a)
                    if hit:
                        out.append(Access(section, kernel, f"arg{ai}", hit[2], a - hit[0], True))
        return out

    def check(self, tag: str = "") -> None:
        """Raise HazardError when the recorded side and main sections conflict."""
        tmap = TensorMap.from_roots(self.roots)
        side, main = self.accesses("side", tmap), self.accesses("main", tmap)
        found = conflicts(side, main, tmap)
        self.checked += 1
        if found:
            lines = [f"  {a!r}  <->  {b!r}" for a, b in found[:20]]
            raise HazardError(f"side/main graph hazard{(' in ' + tag) if tag else ''}: {len(found)} overlapping "
                              "accesses with a write:\n" + "\n".join(lines))


def conflicts(xs: List[Access], ys: List[Access], tmap: Optional[TensorMap] = None) -> List[Tuple[Access, Access]]:
    """Pairs (x, y) whose extents overlap inside one tensor, at least one a write.  An access's
    extent runs from its base to the next base any access uses in the same tensor."""
    bases: Dict[str, List[int]] = defaultdict(list)
    for a in xs + ys:
        bases[a.owner].append(a.base)
    for k in bases:
        bases[k] = sorted(set(bases[k]))

    def extent(a: Access) -> Tuple[int, int]:
        b = bases[a.owner]
        i = bisect.bisect_right(b, a.base)
        return a.base, (b[i] if i < len(b) else 1 << 62)

    out = []
    by_owner = defaultdict(list)
    for y in ys:
        by_owner[y.owner].append(y)
    for x in xs:
        ex = extent(x)
        for y in by_owner.get(x.owner, ()):
            if not (x.write or y.write):
                continue
            ey = extent(y)
            if ex[0] < ey[1] and ey[0] < ex[1]:
                out.append((x, y))
    return out


class HipProxy:
    """The extension module with every launcher call noted by ``rec`` (classes pass through)."""

    def __init__(self, mod, rec: Recorder):
        object.__setattr__(self, "_mod", mod)
        object.__setattr__(self, "_rec", rec)

    def __getattr__(self, name):
        attr = getattr(self._mod, name)
        if isinstance(attr, type) or not callable(attr):
            return attr
        rec = self._rec

        def call(*args, **kwargs):
            rec.note(name, tuple(args) + tuple(kwargs.values()))
            return attr(*args, **kwargs)

        return call


# ---- three-stream plan of the streamed training loop ---------------------------------------------
class StreamPlan:
    """Happens-before checker over the operations of ``FusedDeepFM.train_stream`` on its three
    streams: the copy stream (H2D copies of host batches / raw payloads + the device Example parser
    writing the HBM batch ring), the side stream (each multi-step graph's fetch + sort of the NEXT
    graph's batches — the ring's readers) and the compute stream (the prime, the main graphs).

    The loop records every ``Event.record`` / ``wait_event`` it issues here (``record`` returns a
    token, ``wait`` queues it for the stream's next operation) and every operation with the ring
    slots (or other named ranges) it reads and writes.  Operations on one stream are ordered; across
    streams only through the recorded waits (transitively).  ``check`` raises HazardError for two
    unordered operations whose ranges overlap with at least one write — e.g. a copy that refills a
    ring slot a side graph may still be reading (the event plan's ``copy.wait_event(sevs[j - 3])``).

    Declared ranges are only as good as their annotations: a new write into the ring that the loop
    does not declare would be invisible.  ``ObservedWrites`` closes that for torch ops: while it is
    active every aten op that writes into a registered tensor (the ring) becomes an operation of the
    plan on the stream it was issued on, with the slots it actually touched.  HIP-extension launches
    (the device parser) are not torch ops; they stay declared (and, inside graph capture, observed by
    ``Recorder``).
    """

    def __init__(self, window: int = 96):
        self.ops: List[Tuple[str, str, List[Tuple[str, int, int, bool]], int]] = []  # stream, label, ranges, deps
        self.base = 0  # absolute index of ops[0]: ``check`` prunes to the last ``window`` operations
        self.window = int(window)
        self._last: Dict[str, int] = {}  # stream → absolute index of its last op
        self._waits: Dict[str, int] = defaultdict(int)  # stream → bitmask (relative) of ops its next op waits for

    def record(self, stream: str) -> int:
        """Token of everything issued on ``stream`` so far (an event recorded there): the absolute
        index of its last operation as one bit, valid across pruning."""
        i = self._last.get(stream)
        return 0 if i is None else (1 << i)

    def wait(self, stream: str, token: Optional[int]) -> None:
        if token:
            rel = token >> self.base  # (a token of a pruned op orders nothing left in the window)
            if rel:
                self._waits[stream] |= rel

    def wait_stream(self, stream: str, other: str) -> None:
        self.wait(stream, self.record(other))

    def op(self, stream: str, label: str, ranges=()) -> int:
        """One operation on ``stream``; ``ranges`` = [(name, lo, hi, write)] (half-open)."""
        deps = self._waits.pop(stream, 0)
        last = self._last.get(stream)
        if last is not None and last >= self.base:
            deps |= 1 << (last - self.base)
        i = self.base + len(self.ops)
        self.ops.append((stream, label, list(ranges), deps))
        self._last[stream] = i
        return i

    def prune(self, keep: Optional[int] = None) -> None:
        """Drop all but the last ``keep`` operations.  Exact for the pairs left: happens-before
        edges only point to older operations, so every path between two kept operations runs
        through kept operations.  With ``keep`` above the ring's reuse distance in operations (a
        slot is rewritten every 4 graphs ≈ 16 operations) every access a refill could race is still
        checked, and ``ROCFM_HAZARD=1`` stays O(keep²) per check over a whole epoch."""
        keep = self.window if keep is None else int(keep)
        d = len(self.ops) - keep
        if d <= 0:
            return
        self.ops = [(st, lb, rg, deps >> d) for st, lb, rg, deps in self.ops[d:]]
        for k in list(self._waits):
            self._waits[k] >>= d
        self.base += d

    def conflicts(self) -> List[Tuple[str, str, str]]:
        # transitive happens-before: hb[i] = bitmask of every op ordered before op i
        hb: List[int] = []
        for _, _, _, deps in self.ops:
            m = deps
            d = deps
            while d:
                j = (d & -d).bit_length() - 1
                m |= hb[j]
                d &= d - 1
            hb.append(m)
        out = []
        by_name: Dict[str, List[Tuple[int, int, int, bool]]] = defaultdict(list)
        for i, (_, _, ranges, _) in enumerate(self.ops):
            for name, lo, hi, w in ranges:
                by_name[name].append((i, lo, hi, w))
        for name, acc in by_name.items():
            for a in range(len(acc)):
                i, lo, hi, w = acc[a]
                for b in range(a + 1, len(acc)):
                    j, lo2, hi2, w2 = acc[b]
                    if i == j or not (w or w2) or not (lo < hi2 and lo2 < hi):
                        continue
                    if self.ops[i][0] == self.ops[j][0]:
                        continue  # same stream: ordered
                    x, y = (i, j) if i < j else (j, i)
                    if not (hb[y] >> x) & 1:
                        out.append((name, f"{self.ops[x][0]}:{self.ops[x][1]}", f"{self.ops[y][0]}:{self.ops[y][1]}"))
        return out

    def check(self, tag: str = "") -> None:
        found = self.conflicts()
        if found:
            lines = [f"  {n}: {a}  <->  {b}" for n, a, b in found[:20]]
            raise HazardError(f"stream-plan hazard{(' in ' + tag) if tag else ''}: {len(found)} unordered "
                              "overlapping accesses with a write:\n" + "\n".join(lines))
        self.prune()


# ---- observed writes: torch ops into registered tensors become plan operations ----------------------
class ObservedWrites:
    """Context manager: while active, every aten op writing (in place, or through ``out=``) into a
    registered tensor is recorded in ``plan`` as an operation on the stream it was issued on
    (``stream_of()`` → plan stream name; default: the current CUDA stream through ``names``, a map of
    ``cuda_stream`` handles), with the range it touched in the tensor's leading-dimension units.

    ``tensors`` = {range name: [tensors]}: e.g. ``{"ring": [ids, vals, labels]}`` — every tensor of
    a name shares the slot numbering of its leading dimension, as the plan's declared ranges do.
    ``plan`` and ``tensors`` may be callables, resolved at each write (the engine creates its plan
    and ring inside the loop this wraps); a ``None`` plan records nothing."""

    def __init__(self, plan, tensors, names=None, stream_of=None):
        from torch.utils._python_dispatch import TorchDispatchMode

        self._plan = plan if callable(plan) else (lambda: plan)
        self._tensors = tensors if callable(tensors) else (lambda: tensors)
        names = names or {}
        if stream_of is None:
            def stream_of():
                return names.get(torch.cuda.current_stream().cuda_stream, "?")
        self.stream_of = stream_of
        self.seen = 0
        outer = self

        class _Mode(TorchDispatchMode):
            def __torch_dispatch__(self, func, types, args=(), kwargs=None):
                kwargs = kwargs or {}
                out = func(*args, **kwargs)
                outer._note(func, args, kwargs)
                return out

        self._mode = _Mode()

    def _written(self, func, args, kwargs):
        schema = func._schema
        for i, a in enumerate(schema.arguments):
            if a.alias_info is None or not a.alias_info.is_write:
                continue
            v = args[i] if i < len(args) else kwargs.get(a.name)
            if isinstance(v, torch.Tensor):
                yield v
            elif isinstance(v, (list, tuple)):
                yield from (x for x in v if isinstance(x, torch.Tensor))

    def _regions(self):
        out = []  # (lo byte, hi byte, unit bytes, name)
        for name, ts in (self._tensors() or {}).items():
            for t in ts:
                if t is not None and t.numel():
                    lo = t.data_ptr()
                    out.append((lo, lo + t.numel() * t.element_size(), t.stride(0) * t.element_size(), name))
        return out

    def _note(self, func, args, kwargs) -> None:
        plan = self._plan()
        if plan is None:
            return
        regions = self._regions()
        ranges = []
        for t in self._written(func, args, kwargs):
            if t.numel() == 0:
                continue
            a = t.data_ptr()
            e = a + t.numel() * t.element_size()  # (a contiguous view: the ring's slot slices are)
            for lo, hi, unit, name in regions:
                if a < hi and lo < e:
                    s0 = (max(a, lo) - lo) // unit
                    s1 = (min(e, hi) - lo + unit - 1) // unit
                    ranges.append((name, int(s0), int(s1), True))
        if ranges:
            self.seen += 1
            plan.op(self.stream_of(), f"observed {func}", ranges)

    def __enter__(self):
        self._mode.__enter__()
        return self

    def __exit__(self, *exc):
        return self._mode.__exit__(*exc)
