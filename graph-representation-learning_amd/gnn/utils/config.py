"""YAML config -> attribute-access dict.

The reference loads configs with anyconfig + munch (gnn/cl_warper.py:61-79);
neither is installed here, so this is a minimal equivalent: yaml.safe_load
(no object construction) and a recursive dict subclass with attribute
access.  Missing keys read as None through attribute access, like
munch.DefaultMunch would not -- we follow munch: AttributeError.
"""
from __future__ import annotations

from typing import Any

import yaml


class AttrDict(dict):
    """dict with attribute access, recursively applied to nested dicts/lists."""

    def __init__(self, *args, **kwargs):
        super().__init__(*args, **kwargs)
        for k, v in list(self.items()):
            super().__setitem__(k, _wrap(v))

    def __getattr__(self, name: str) -> Any:
        try:
            return self[name]
        except KeyError as err:
            raise AttributeError(name) from err

    def __setattr__(self, name: str, value: Any) -> None:
        self[name] = value

    def __setitem__(self, key, value) -> None:
        super().__setitem__(key, _wrap(value))

    def __delattr__(self, name: str) -> None:
        try:
            del self[name]
        except KeyError as err:
            raise AttributeError(name) from err

    def get(self, key, default=None):  # keep dict semantics
        return super().get(key, default)


def _wrap(v: Any) -> Any:
    if isinstance(v, dict) and not isinstance(v, AttrDict):
        return AttrDict(v)
    if isinstance(v, list):
        return [_wrap(x) for x in v]
    return v


def to_plain(v: Any) -> Any:
    """AttrDict tree -> plain dict/list tree (safe for torch.save with
    weights_only loading, unlike the reference's munch config)."""
    if isinstance(v, dict):
        return {k: to_plain(x) for k, x in v.items()}
    if isinstance(v, (list, tuple)):
        return [to_plain(x) for x in v]
    return v


def load_config(path: str) -> AttrDict:
    with open(path, encoding="utf-8-sig") as f:
        return AttrDict(yaml.safe_load(f) or {})


def node_range_parallel(cfg) -> bool:
    """Additive config key `graph_parallel`: "node_range" (with distributed:
    true) trains and validates every batch's graph as node-range shards, one
    per rank (grl.dist.ShardedGraph), instead of the reference's data
    parallelism over documents; absent / "documents" keeps the latter."""
    v = cfg.get("graph_parallel")
    if v in (None, False, "", "none", "documents"):
        return False
    if v != "node_range":
        raise ValueError(f"graph_parallel must be 'node_range' or 'documents', got {v!r}")
    return bool(cfg.get("distributed"))
