"""Cassia-format documents: a list of {"location": 4 points, "text", ...}
(the reference's CassiaDataset, datasets/cassia_dataset.py:11-247); the
format predict() receives."""
from typing import Any, Dict, List

from gnn.data_generator.datasets.base_dataset import DocumentDataset


class CassiaDataset(DocumentDataset):
    def _load_annotations(self, sample: List[Dict[str, Any]]) -> Dict[int, Dict[str, Any]]:
        out: Dict[int, Dict[str, Any]] = {}
        for idx, region in enumerate(sample):
            region["polygon"] = region["location"]
            out[idx] = region
        return out
