"""Synthetic Criteo-shape data (39 fields) with the layout of the bundled data.

The bundled ``data/val.tfrecords`` has 13 numeric fields carrying fixed ids 1..13 and
real values, then 26 categorical fields with value 1.0 and ids in disjoint per-field ranges.  This
generator reproduces that layout for any vocabulary size ``V``:

* categorical field f gets ``min(card_f, cap)`` ids (Criteo-Kaggle cardinalities, capped so the
  fields exactly fill ``[14, V)`` — "hashing into a V-row vocabulary");
* ids are drawn per field from a Zipf(α) law over the field's range (rank r → id via a fixed
  stride permutation), so batches show the hot-row skew of real CTR data;
* labels come from a fixed random logistic "teacher" over the same ids, so a model can learn
  (AUC well above 0.5) and ≈25 % of examples are positive like the bundled data.

Generation runs on whatever device is asked for (the benchmark builds an HBM-resident dataset).
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import List, Optional, Tuple

import numpy as np
import torch

CRITEO_CARDINALITIES = [1460, 583, 10131227, 2202608, 305, 24, 12517, 633, 3, 93145, 5683, 8351593, 3194, 27,
                        14992, 5461306, 10, 5652, 2173, 4, 7046547, 18, 15, 286181, 105, 142572]
NUM_NUMERIC = 13


def field_sizes(vocab: int, n_cat: int = 26) -> List[int]:
    """Per-categorical-field id counts filling [NUM_NUMERIC+1, vocab)."""
    avail = vocab - (NUM_NUMERIC + 1)
    cards = (CRITEO_CARDINALITIES * ((n_cat + 25) // 26))[:n_cat]
    if avail < n_cat:
        raise ValueError(f"vocabulary {vocab} too small for {n_cat} categorical fields")
    if sum(cards) <= avail:
        sizes = list(cards)
    else:
        lo, hi = 1, max(cards)
        while lo < hi:  # largest cap with Σ min(card, cap) <= avail
            mid = (lo + hi + 1) // 2
            if sum(min(c, mid) for c in cards) <= avail:
                lo = mid
            else:
                hi = mid - 1
        sizes = [min(c, lo) for c in cards]
        # hand the remainder to the capped fields
        rem = avail - sum(sizes)
        i = 0
        while rem > 0:
            if cards[i % n_cat] > sizes[i % n_cat]:
                sizes[i % n_cat] += 1
                rem -= 1
            i += 1
    return sizes


@dataclass
class SyntheticCriteo:
    vocab: int
    field_size: int = 39
    zipf_alpha: float = 1.1
    seed: int = 0
    positive_rate: float = 0.255

    def __post_init__(self):
        if self.field_size < NUM_NUMERIC + 1:
            raise ValueError("field_size must be >= 14 (13 numeric + categorical)")
        self.n_cat = self.field_size - NUM_NUMERIC
        self.sizes = field_sizes(self.vocab, self.n_cat)
        self.offsets = np.cumsum([NUM_NUMERIC + 1] + self.sizes[:-1]).tolist()
        rng = np.random.default_rng(self.seed + 7919)
        # teacher weights: numeric fields + a sparse set of strong categorical ids
        self.teacher_num = rng.normal(0.0, 0.6, NUM_NUMERIC).astype(np.float32)
        self.teacher_seed = self.seed + 104729
        self._cdf_cache = {}

    def _cdf(self, size: int, device) -> torch.Tensor:
        key = (size, str(device))
        if key not in self._cdf_cache:
            n = min(size, 1 << 22)
            w = (np.arange(1, n + 1, dtype=np.float64)) ** (-self.zipf_alpha)
            c = np.cumsum(w)
            c /= c[-1]
            self._cdf_cache[key] = torch.from_numpy(c.astype(np.float64)).to(device)
        return self._cdf_cache[key]

    def _teacher_w(self, ids: torch.Tensor) -> torch.Tensor:
        """Deterministic pseudo-random teacher weight per id (hash), ~N(0,1)-ish, sparse."""
        h = (ids.to(torch.int64) * 2654435761 + self.teacher_seed) % 2147483647
        h = (h * 48271) % 2147483647
        u = h.to(torch.float64) / 2147483647.0
        w = torch.where(u < 0.15, (u / 0.15 - 0.5) * 4.0, torch.zeros_like(u))
        return w.to(torch.float32)

    def batch(self, n: int, device="cpu", gen: Optional[torch.Generator] = None
              ) -> Tuple[torch.Tensor, torch.Tensor, torch.Tensor]:
        """(ids int32 [n,F], vals f32 [n,F], labels f32 [n])."""
        dev = torch.device(device)
        if gen is None:
            gen = torch.Generator(device=dev).manual_seed(self.seed)
        F = self.field_size
        ids = torch.empty(n, F, dtype=torch.int64, device=dev)
        vals = torch.ones(n, F, dtype=torch.float32, device=dev)
        ids[:, :NUM_NUMERIC] = torch.arange(1, NUM_NUMERIC + 1, device=dev)
        # numeric values: many zeros, log-scaled magnitudes (like the bundled data's 0..145 range)
        z = torch.rand(n, NUM_NUMERIC, generator=gen, device=dev)
        mag = torch.rand(n, NUM_NUMERIC, generator=gen, device=dev)
        vals[:, :NUM_NUMERIC] = torch.where(z < 0.35, torch.zeros_like(mag), (mag * 3.0).exp_() * 0.05)
        for j in range(self.n_cat):
            size = self.sizes[j]
            cdf = self._cdf(size, dev)
            u = torch.rand(n, generator=gen, device=dev, dtype=torch.float64)
            rank = torch.searchsorted(cdf, u).clamp_(max=cdf.numel() - 1)
            if size > cdf.numel():  # tail beyond the tabulated CDF: spread uniformly
                tail = torch.randint(0, size, (n,), generator=gen, device=dev)
                rank = torch.where(rank == cdf.numel() - 1, tail, rank)
            stride = 1000003 % size if size > 1 else 1
            if math.gcd(stride, size) != 1:
                stride = 1
            ids[:, NUM_NUMERIC + j] = self.offsets[j] + (rank * stride) % size
        tw = self._teacher_w(ids)
        tn = torch.from_numpy(self.teacher_num).to(dev)
        logit = (tw[:, NUM_NUMERIC:] * vals[:, NUM_NUMERIC:]).sum(1) + (vals[:, :NUM_NUMERIC] * tn).sum(1) * 0.3
        logit = logit - 1.6
        labels = (torch.rand(n, generator=gen, device=dev) < torch.sigmoid(logit)).to(torch.float32)
        return ids.to(torch.int32), vals, labels


def write_synthetic_tfrecord(path: str, n: int, vocab: int, field_size: int = 39, seed: int = 0,
                             chunk: int = 65536) -> int:
    """Write ``n`` synthetic examples as a TFRecord file (C++ writer)."""
    from ..ops import require_io

    io = require_io()
    gen_ = SyntheticCriteo(vocab, field_size, seed=seed)
    g = torch.Generator().manual_seed(seed)
    done = 0
    while done < n:
        m = min(chunk, n - done)
        ids, vals, labels = gen_.batch(m, "cpu", g)
        io.write_tfrecord(path, labels.numpy(), ids.numpy().astype(np.int64), vals.numpy(), done > 0)
        done += m
    io.build_index(path, True)  # the persistent record index next to the file (record_index.h)
    return done
