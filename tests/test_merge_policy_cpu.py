"""DP merge policy (no GPU): which worlds take the directory-narrowed search merge."""
from rocfm.parallel.dp import SEARCH_DIR_MAX_W, search_dir_buckets


def test_search_dir_buckets_policy(monkeypatch):
    monkeypatch.delenv("ROCFM_SEARCH_DIR", raising=False)
    monkeypatch.delenv("ROCFM_MERGE", raising=False)
    assert SEARCH_DIR_MAX_W == 4
    assert search_dir_buckets(1, 1_000_000) == 0  # one rank never merges
    assert search_dir_buckets(2, 1_000_000) == 8192 and search_dir_buckets(4, 1_000_000) == 8192
    assert search_dir_buckets(8, 1_000_000) == 0  # the maps merge beyond 4 ranks
    assert search_dir_buckets(2, 20_000) == 1250 and search_dir_buckets(2, 500) == 64  # ≥ 16 ids per bucket, ≥ 64
    monkeypatch.setenv("ROCFM_SEARCH_DIR", "0")
    assert search_dir_buckets(2, 1_000_000) == 0
    monkeypatch.setenv("ROCFM_SEARCH_DIR", "1")
    for forced in ("direct", "hash", "range"):  # a forced merge mode keeps its own path
        monkeypatch.setenv("ROCFM_MERGE", forced)
        assert search_dir_buckets(2, 1_000_000) == 0


def test_plan_merge_policy(monkeypatch):
    """The plan-ahead merge: the default with the p2p exchange from PLAN_MIN_W (5) ranks; over RCCL
    only when forced (ROCFM_MERGE=plan); any other forced merge keeps it off; one rank never."""
    from rocfm.parallel.dp import PLAN_MIN_W, plan_merge_enabled
    monkeypatch.delenv("ROCFM_MERGE", raising=False)
    assert PLAN_MIN_W == 5
    assert not plan_merge_enabled(1, "p2p")
    assert not plan_merge_enabled(4, "p2p") and plan_merge_enabled(8, "p2p")
    assert not plan_merge_enabled(8, "rccl")
    monkeypatch.setenv("ROCFM_MERGE", "plan")
    assert plan_merge_enabled(2, "rccl") and not plan_merge_enabled(1, "rccl")
    for m in ("direct", "hash", "range"):
        monkeypatch.setenv("ROCFM_MERGE", m)
        assert not plan_merge_enabled(8, "p2p")
