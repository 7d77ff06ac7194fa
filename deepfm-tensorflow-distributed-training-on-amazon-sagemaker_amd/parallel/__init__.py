"""Distributed training: data parallel (dp), row-sharded embeddings (emb_shard), the p2p xGMI exchange, self-validation."""
