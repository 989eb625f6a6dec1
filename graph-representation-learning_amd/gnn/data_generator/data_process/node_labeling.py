"""Class index of each text line: class_to_id[formal_key][key_type], 0 for
anything unlabelled (the reference's NodeLabeling, data_process/node_labeling.py)."""
from typing import Any, Dict

import numpy as np

from gnn.data_generator.data_process.base import BaseDataProcess


class NodeLabeling(BaseDataProcess):
    def __init__(self):
        pass

    def process(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        if sample.get("label", None) is None:
            return sample
        class_to_id = sample["class_to_id"]
        sample["node_label"] = np.array(
            [class_to_id.get(t.get("label"), {}).get(t.get("key_type"), 0) for t in self.ordered_lines(sample)])
        return sample
