"""One-shot xGMI push exchange over IPC-mapped peer buffers (csrc/kernels/p2p.hip).

SURVEY §5.8 item 2 / N14 / §7.2 P6.  The DP step exchanges ≈1 MB per rank per step (MLP
gradients + compacted embedding rows, ``rocfm.parallel.dp``).  RCCL's all-gather of that bucket is
latency-bound: on one node of fully connected xGMI a ring needs W−1 dependent hops.  Here every
rank maps every other rank's receive buffer and flag block once (``hipIpcGetMemHandle`` /
``hipIpcOpenMemHandle``, handles exchanged over the process group), and ONE kernel pushes the
payload to all peers at once — W−1 links, one hop each — with a flag hand-off instead of a
collective protocol.  The launch advances its own device-side exchange counter, so it is captured
into the multi-step HIP graphs like any other kernel (also when the process group is gloo).

Receive buffers and flags are allocated uncached (``hipDeviceMallocUncached``) so that a peer's
writes are visible to the kernels that read them next without any L2 maintenance.  Every wait in
the kernel is bounded: a peer that never arrives raises a sticky error flag (``errored()``)
instead of hanging the GPU.  The default bound (2^30 polls, about a minute) only fires when a
peer is gone: ranks that stall on host work (rank 0 writing a checkpoint) are drained and joined
by a barrier first (Estimator._save), so healthy peers never wait that long.

The reference has no equivalent: Horovod hands the gradients to NCCL (HVD:296).
"""
from __future__ import annotations

import logging
import math
import os
from typing import List, Optional, Tuple

import torch
import torch.distributed as dist

KIND_UNCACHED, KIND_FINEGRAINED, KIND_PLAIN = 0, 1, 2
log = logging.getLogger("rocfm")


def _pci_key(dev: torch.device) -> Tuple[int, int, int]:
    pr = torch.cuda.get_device_properties(dev)
    return (int(pr.pci_domain_id), int(pr.pci_bus_id), int(pr.pci_device_id))


def peer_access_problem(device, keys: List[Tuple[int, int, int]], rank: int) -> Optional[str]:
    """Why this rank's GPU cannot write into a peer rank's GPU, or None.  ``keys`` are every
    rank's PCI (domain, bus, device).  A peer GPU that is visible in this process is checked with
    hipDeviceCanAccessPeer; a peer on the SAME GPU (ranks sharing a card) needs no peer path; a
    peer GPU this process cannot see (per-rank device masks) is left to the self-test."""
    dev = torch.device(device)
    mine = keys[rank]
    local = {}
    for d in range(torch.cuda.device_count()):
        local[_pci_key(torch.device("cuda", d))] = d
    for r, k in enumerate(keys):
        if r == rank or k == mine or k not in local:
            continue
        if not torch.cuda.can_device_access_peer(dev.index, local[k]):
            return f"GPU {dev.index} cannot access peer GPU {local[k]} (rank {r}): no xGMI/PCIe peer path"
    return None


def _hip():
    from ..ops import hip

    return hip()


def single_node(group=None) -> bool:
    """True when every rank of the group runs on this host (IPC mapping needs one node)."""
    if not dist.is_initialized():
        return True
    lw = os.environ.get("LOCAL_WORLD_SIZE")
    if lw is not None and int(lw) == dist.get_world_size(group):
        return True
    names: List[Optional[str]] = [None] * dist.get_world_size(group)
    dist.all_gather_object(names, os.uname().nodename, group=group)
    return len(set(names)) == 1


class P2PExchange:
    """W receive slots of ``slot_floats`` f32 per rank, mapped into every peer.

    ``push(params)`` launches the exchange on the current stream: destination ``d`` receives
    ``n_floats`` floats from ``src + d * src_stride`` (``src_stride=0``: all-gather) into its
    slot ``rank``.  After the launch completes, ``recv_ptr + r * slot_floats * 4`` holds rank r's
    payload on every rank.
    """

    def __init__(self, slot_floats: int, device, group=None, kind: int = KIND_UNCACHED,
                 spin_limit: Optional[int] = None, extra_floats: int = 0):
        H = self.H = _hip()
        self.group = group
        self.W = dist.get_world_size(group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(group) if dist.is_initialized() else 0
        if self.W > H.p2p_max_world():
            raise ValueError(f"p2p exchange supports at most {H.p2p_max_world()} ranks, got {self.W}")
        self.device = torch.device(device)
        self.slot = (int(slot_floats) + 3) // 4 * 4
        # local floats behind the W slots (never pushed; e.g. the row-shard hot-row replica)
        self.extra = (int(extra_floats) + 3) // 4 * 4
        # polls per wave before a wait gives up and raises the sticky error flag; ROCFM_SPIN_LIMIT
        # lowers it for rehearsals that force producer pushes onto one shared GPU (fail fast, loud)
        self.spin_limit = int(spin_limit if spin_limit is not None else os.environ.get("ROCFM_SPIN_LIMIT", 1 << 30))
        self.kind = kind
        self._own: List[int] = []
        self._opened: List[int] = []
        self.init_error: Optional[BaseException] = None
        self.peers: List[Tuple[int, int]] = []
        # every rank takes part in every collective below even if a step fails on it, so that a
        # local failure becomes an agreed fallback (selftest) instead of a hang
        mine = None
        # ranks sharing one GPU (rehearsals on a one-GPU box): producer-side pushing is unsafe there
        # (a rank's spinning producers can occupy the CUs its lagging peer needs to raise its flag)
        self.shared_device = False
        if self.W > 1:  # peer-access check first (a failure becomes an agreed RCCL fallback below)
            keys: List = [None] * self.W
            dist.all_gather_object(keys, _pci_key(self.device), group=group)
            self.shared_device = len(set(keys)) < self.W
            try:
                why = peer_access_problem(self.device, keys, self.rank)
            except Exception as exc:  # property queries failing: leave the verdict to the self-test
                why = None
                log.debug("p2p peer-access check skipped: %s", exc)
            if why:
                self.init_error = RuntimeError(why)
        with torch.cuda.device(self.device):
            self.ctrl = torch.zeros(2, dtype=torch.int32, device=self.device)   # exchange count, arrivals
            self.error = torch.zeros(1, dtype=torch.int32, device=self.device)
            try:
                if self.init_error is not None:
                    raise self.init_error
                self.recv_ptr = H.p2p_malloc((self.W * self.slot + self.extra) * 4, kind)
                self._own.append(self.recv_ptr)
                self.sig_ptr = H.p2p_malloc(max(256, 8 * self.W), kind)
                self._own.append(self.sig_ptr)
                mine = (H.p2p_ipc_handle(self.recv_ptr), H.p2p_ipc_handle(self.sig_ptr))
            except Exception as exc:
                self.init_error = exc
            handles: List[Optional[Tuple[bytes, bytes]]] = [mine]
            if self.W > 1:
                handles = [None] * self.W
                dist.all_gather_object(handles, mine, group=group)
            if any(h is None for h in handles):
                self.init_error = self.init_error or RuntimeError("p2p buffer setup failed on a peer")
            else:
                try:
                    for r in range(self.W):
                        if r == self.rank:
                            self.peers.append((self.recv_ptr, self.sig_ptr))
                            continue
                        a = H.p2p_ipc_open(handles[r][0])
                        self._opened.append(a)
                        b = H.p2p_ipc_open(handles[r][1])
                        self._opened.append(b)
                        self.peers.append((a, b))
                except Exception as exc:
                    self.init_error = exc
        if self.W > 1:
            dist.barrier(group=group)  # every rank's buffers are zeroed and mapped before any push

    def params(self, src_ptr: int, n_floats: int, src_stride_floats: int = 0, chunks: Optional[int] = None,
               spin_limit: Optional[int] = None, dst_offset_floats: int = 0):
        """Push parameters.  ``dst_offset_floats``: the payload lands that far into each slot (a
        fused-push exchange publishes only the part its producers did not store themselves)."""
        if n_floats % 4 or src_stride_floats % 4 or src_ptr % 16 or dst_offset_floats % 4:
            raise ValueError("p2p payloads must be whole, 16-byte aligned float4 runs")
        if n_floats + dst_offset_floats > self.slot:
            raise ValueError(f"payload of {n_floats} floats at {dst_offset_floats} exceeds the {self.slot}-float slot")
        p = self.H.P2PParams()
        p.src = src_ptr
        p.n4 = n_floats // 4
        p.src_stride4 = src_stride_floats // 4
        p.slot4 = self.slot // 4
        for r, (a, b) in enumerate(self.peers):
            p.set_peer(r, a + 4 * dst_offset_floats, b)
        p.ctrl = self.ctrl.data_ptr()
        p.error = self.error.data_ptr()
        p.W, p.rank = self.W, self.rank
        # ≈16 KiB per workgroup, ≤64 chunks per destination (≤1024 workgroups at W=16)
        p.chunks = int(chunks or max(1, min(64, math.ceil(n_floats * 4 / 16384))))
        p.spin_limit = int(spin_limit or self.spin_limit)
        return p

    def push_target(self):
        """Producer-side push into this exchange (csrc/kernels/push.h): this rank's slot in every
        rank's receive buffer, the peers' flag blocks, the exchange counter and error flag."""
        if self.W > self.H.push_max_world():
            raise ValueError(f"fused push supports at most {self.H.push_max_world()} ranks, got {self.W}")
        t = self.H.PushTarget()
        t.W, t.rank = self.W, self.rank
        for d, (recv, sig) in enumerate(self.peers):
            t.set_dest(d, recv + self.rank * self.slot * 4, sig)
        t.ctrl = self.ctrl.data_ptr()
        t.error = self.error.data_ptr()
        t.spin_limit = self.spin_limit
        return t

    def push(self, p, stream: Optional[int] = None) -> None:
        if stream is None:
            stream = torch.cuda.current_stream(self.device).cuda_stream
        self.H.p2p_push(p, stream)

    @staticmethod
    def push_multi(exs: List["P2PExchange"], ps, stream: Optional[int] = None) -> None:
        """Hand off several distinct exchanges (``ps[i]`` built by ``exs[i].params``) in ONE launch:
        each keeps its own flags and counters, and their peer waits overlap (p2p.hip
        p2p_push_multi_kernel).  Every rank must combine the same exchanges in the same launch."""
        if len(exs) == 1:
            exs[0].push(ps[0], stream)
            return
        if stream is None:
            stream = torch.cuda.current_stream(exs[0].device).cuda_stream
        exs[0].H.p2p_push_multi(list(ps), stream)

    def slot_ptr(self, r: int) -> int:
        return self.recv_ptr + r * self.slot * 4

    def copy_out(self, out: torch.Tensor) -> torch.Tensor:
        """Copy the W receive slots into ``out`` ([W * slot] f32, same device) on the current stream."""
        if out.numel() < self.W * self.slot or out.dtype != torch.float32 or not out.is_contiguous():
            raise ValueError("copy_out needs a contiguous f32 tensor of W*slot elements")
        self.H.memcpy_d2d(out.data_ptr(), self.recv_ptr, self.W * self.slot * 4,
                          torch.cuda.current_stream(self.device).cuda_stream)
        return out

    def recv_tensor(self, dtype: torch.dtype, shape) -> torch.Tensor:
        """The W receive slots as a torch tensor (no copy; 4-byte dtypes, ≤ W·slot elements).
        The tensor borrows the buffer: keep this exchange open while it is used."""
        if torch.empty(0, dtype=dtype).element_size() != 4:
            raise ValueError("recv_tensor supports 4-byte dtypes")
        n = int(math.prod(shape))
        if n > self.W * self.slot + self.extra:
            raise ValueError(f"{n} elements exceed the {self.W}x{self.slot} receive slots (+{self.extra})")
        typestr = {torch.float32: "<f4", torch.int32: "<i4"}[dtype]

        class _Raw:  # __cuda_array_interface__ v3 view of the uncached HIP allocation
            pass

        raw = _Raw()
        raw.__cuda_array_interface__ = {"shape": (n,), "typestr": typestr, "data": (self.recv_ptr, False),
                                        "version": 3, "strides": None}
        return torch.as_tensor(raw, device=self.device).view(*shape)

    def clear(self) -> None:
        """Zero this rank's W receive slots (e.g. the self-test's patterns) and wait until every
        rank has done so, so no peer's next push can land before the clear.  Collective."""
        self.recv_tensor(torch.float32, (self.W * self.slot,)).zero_()
        torch.cuda.synchronize(self.device)
        if self.W > 1 and dist.is_initialized():
            dist.barrier(group=self.group)

    def errored(self) -> bool:
        return bool(int(self.error.item()))

    def close(self) -> None:
        """Unmap the peers' buffers and free this rank's (call on every rank, GPU idle)."""
        if getattr(self, "_closed", False):
            return
        self._closed = True  # set on every rank: the barriers below are matched
        torch.cuda.synchronize(self.device)
        if self.W > 1 and dist.is_initialized():
            dist.barrier(group=self.group)  # no peer still writes into our buffers
        with torch.cuda.device(self.device):
            for a in self._opened:
                self.H.p2p_ipc_close(a)
            if self.W > 1 and dist.is_initialized():
                dist.barrier(group=self.group)  # every peer has unmapped ours before we free it
            for a in self._own:
                self.H.p2p_free(a)
        self._own, self._opened = [], []


def producer_push_enabled(ex) -> bool:
    """Whether an exchange's producers push into the peers' slots themselves (csrc/kernels/push.h).
    ``ROCFM_DP_PUSH``: ``auto`` (default) — yes, unless ranks share a GPU (one-box rehearsals: a
    rank's spinning producers could hold the CUs a lagging peer needs to raise its flag); ``1`` —
    force (small test batches on a shared GPU); ``0`` — never (the push launch copies the bucket).
    At most ``push_max_world()`` ranks (one node)."""
    mode = os.environ.get("ROCFM_DP_PUSH", "auto").lower()
    if mode not in ("auto", "0", "1"):
        raise ValueError(f"ROCFM_DP_PUSH must be auto, 0 or 1, got {mode!r}")
    if ex.W > ex.H.push_max_world():
        return False
    return mode == "1" or (mode == "auto" and not ex.shared_device)


def selftest(ex: P2PExchange, n_floats: int, rounds: int = 3) -> bool:
    """Push rank-tagged patterns through ``ex`` and check every slot on every rank.  Returns the
    agreement of all ranks (every rank returns the same value)."""
    dev = ex.device
    ok = ex.init_error is None
    try:
        if not ok:
            raise RuntimeError("p2p setup failed")
        n = max(4, n_floats // 4 * 4)
        src = torch.empty(n, dtype=torch.float32, device=dev)
        out = torch.empty(ex.W * ex.slot, dtype=torch.float32, device=dev)
        idx = torch.arange(n, dtype=torch.float32, device=dev)
        p = ex.params(src.data_ptr(), n, spin_limit=1 << 24)  # ≈1 s: a missing peer fails fast here
        for it in range(rounds):
            src.copy_(idx * 0.5 + (1000.0 * ex.rank + 7.0 * it))
            ex.push(p)
            ex.copy_out(out)
            got = out.view(ex.W, ex.slot)[:, :n]
            want = idx.unsqueeze(0) * 0.5 + (1000.0 * torch.arange(ex.W, device=dev).unsqueeze(1) + 7.0 * it)
            ok = ok and bool(torch.equal(got, want))
        ok = ok and not ex.errored()
    except Exception:  # a mapping / launch failure on this rank: agree on the fallback below
        ok = False
    if ex.W > 1 and dist.is_initialized():
        flag = torch.tensor([1 if ok else 0], dtype=torch.int32,
                            device=dev if dist.get_backend(ex.group) == "nccl" else "cpu")
        dist.all_reduce(flag, op=dist.ReduceOp.MIN, group=ex.group)
        ok = bool(int(flag.item()))
    return ok


def open_exchanges(slot_floats: List[int], device, choice: Optional[str] = None,
                   extra_floats: Optional[List[int]] = None) -> Optional[List[P2PExchange]]:
    """One P2PExchange per slot size, or None for the RCCL path.

    ``choice`` (default: env ROCFM_DP_EXCHANGE, else ``auto``): ``rccl`` → None; ``p2p`` → the
    exchanges or an error; ``auto`` → the exchanges when there is more than one rank, every rank
    is on this node and the self-test of every exchange passes on every rank (agreed), else None.
    Collective: every rank of the default group must call it with the same arguments."""
    choice = (choice or os.environ.get("ROCFM_DP_EXCHANGE", "auto")).lower()
    if choice not in ("auto", "p2p", "rccl"):
        raise ValueError(f"exchange must be auto, p2p or rccl, got {choice!r}")
    world = dist.get_world_size() if dist.is_initialized() else 1
    if world == 1 or choice == "rccl":
        return None
    if not single_node():
        if choice == "p2p":
            raise RuntimeError("exchange=p2p needs every rank on one node")
        return None
    extra = list(extra_floats or [0] * len(slot_floats))
    exs = [P2PExchange(n, device, extra_floats=x) for n, x in zip(slot_floats, extra)]  # collective
    ok = True
    for ex, n in zip(exs, slot_floats):
        ok = selftest(ex, n) and ok  # every rank runs every self-test (each one is agreed)
    if ok:
        # slots start zeroed: a fused-push producer (rocfm.parallel.dp) never writes the padding
        # words of its slot, which the MLP optimizer still reads
        for ex in exs:
            ex.clear()
        log.info("exchange: p2p push over IPC-mapped peer buffers (%d ranks, self-test passed)", world)
        return exs
    err = next((ex.init_error for ex in exs if ex.init_error is not None), None)
    for ex in exs:
        ex.close()
    if choice == "p2p":
        raise RuntimeError(f"p2p exchange unavailable: {err or 'self-test failed'}")
    reason = f"{err}" if err else "self-test failed on some rank"
    log.warning("exchange: falling back to RCCL (p2p unavailable: %s)", reason)
    if dist.get_rank() == 0:
        print(f"[rocfm] exchange: falling back to RCCL (p2p unavailable: {reason})", flush=True)
    return None
