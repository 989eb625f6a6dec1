"""Dataset + collate -> torch DataLoader (the reference's BaseDataLoader,
gnn/data_generator/base_dataloader.py:13-112): same config keys, the
collate chain Compose[configured collates..., default_collate], DistributedSampler
when config.distributed (not with graph_parallel: node_range, where every rank
loads the same batches)."""
from __future__ import annotations

import logging
from typing import Any, Callable, Dict, List

import torch
from torch.utils.data import DataLoader
from torch.utils.data._utils.collate import default_collate
from torch.utils.data.distributed import DistributedSampler

from gnn.data_generator import data_collate, datasets
from gnn.data_generator.data_collate.numpy_padding import TypedEdgePadding
from gnn.utils.config import node_range_parallel


def _to_tensors(batch: Dict[str, Any]) -> Dict[str, Any]:
    return {k: torch.from_numpy(v) if hasattr(v, "dtype") and not isinstance(v, torch.Tensor) else v
            for k, v in batch.items()}


class Compose:
    def __init__(self, fns: List[Callable]):
        self.fns = fns

    def __call__(self, x):
        for fn in self.fns:
            x = fn(x)
        return x


class BaseDataLoader:
    def __init__(self, config: Dict[str, Any]):
        self.config = config
        self.logger = logging.getLogger(__name__)

    @classmethod
    def _from_config(cls, config_path: str) -> "BaseDataLoader":
        from gnn.utils.config import load_config

        return cls(load_config(config_path))

    def _load_collate_processors(self, collate_config: Dict[str, Any]) -> List[Callable]:
        procs: List[Callable] = []
        for name, args in (collate_config or {}).items():
            procs.append(getattr(data_collate, name)._from_config(args))
        # TypedEdgePadding already emits one batched dict; others go through default_collate
        procs.append(_to_tensors if any(isinstance(p, TypedEdgePadding) for p in procs) else default_collate)
        return procs

    def _load_dataset(self, dataset_type: str, args: Dict[str, Any], **kwargs) -> datasets.BaseDataset:
        cls = getattr(datasets, dataset_type, None)
        if cls is None:
            raise KeyError(f"Cannot find dataset {dataset_type}")
        return cls._from_config(args, **kwargs)

    def _get_dataloader(self, dataset, data_config: Dict[str, Any], custom_collate: Callable = None,
                        **kwargs) -> DataLoader:
        try:
            collate = Compose(self._load_collate_processors(data_config.get("data_collate")))
            # graph_parallel node_range (additive): every rank loads the same batches and takes a node range
            # of each batch's graph, so no document sampler
            distributed = bool(self.config.get("distributed")) and not node_range_parallel(self.config)
            batch_size = data_config.get("batch_size", 1)
            sampler = None
            if distributed:
                # the initialised process group is the truth for replicas and rank (config.num_gpus /
                # local_rank only stand in before it exists); a different count would overlap or
                # skip documents
                if torch.distributed.is_available() and torch.distributed.is_initialized():
                    replicas, rank = torch.distributed.get_world_size(), torch.distributed.get_rank()
                else:
                    replicas, rank = int(self.config.num_gpus), int(self.config.local_rank)
                batch_size = max(1, batch_size // replicas)  # the reference can reach 0 here
                sampler = DistributedSampler(dataset, num_replicas=replicas, rank=rank,
                                             shuffle=bool(data_config.get("shuffle")))
            elif node_range_parallel(self.config) and bool(data_config.get("shuffle")):
                # node_range: every rank must see the SAME batch each step, so the config's shuffle runs as
                # one replica's sampler with a fixed seed on every rank (set_epoch reshuffles per epoch)
                sampler = DistributedSampler(dataset, num_replicas=1, rank=0, shuffle=True, drop_last=False)
            return DataLoader(dataset, batch_size=batch_size, num_workers=data_config.get("num_workers", 0),
                              drop_last=bool(data_config.get("drop_last")),
                              pin_memory=bool(data_config.get("pin_memory")) and torch.cuda.is_available(),
                              collate_fn=custom_collate if custom_collate is not None else collate,
                              shuffle=False, sampler=sampler)
        except Exception as err:
            self.logger.error(err)
            raise ValueError(err)
