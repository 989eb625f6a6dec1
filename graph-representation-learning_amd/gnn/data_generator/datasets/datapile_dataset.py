"""Datapile (VIA) labelled documents (the reference's DatapileDataset,
datasets/datapile_dataset.py:10-276)."""
from typing import Any, Dict

from gnn.data_generator.datasets.base_dataset import DocumentDataset


class DatapileDataset(DocumentDataset):
    def _load_annotations(self, sample: Dict[str, Any]) -> Dict[int, Dict[str, Any]]:
        """VIA regions -> {region index: {polygon, text, label, key_type}};
        regions without text are skipped (indices keep their gaps)."""
        try:
            regions = sample["attributes"]["_via_img_metadata"]["regions"]
        except KeyError:
            regions = None
            for item in sample.values():  # plain VIA project: {image key: {"regions": [...]}} (last wins)
                regions = item["regions"]
        out: Dict[int, Dict[str, Any]] = {}
        for idx, region in enumerate(regions or []):
            attr, shape = region["region_attributes"], region["shape_attributes"]
            try:
                if shape["name"] == "polygon":
                    polygon = list(zip(shape["all_points_x"], shape["all_points_y"]))
                else:
                    x1, y1 = shape["x"], shape["y"]
                    x2, y2 = shape["width"] + x1, shape["height"] + y1
                    polygon = [(x1, y1), (x2, y1), (x2, y2), (x1, y2)]
            except KeyError as err:
                self.logger.error(err)
                continue
            text = str(attr.get("label", ""))
            if text:
                out[idx] = {"polygon": polygon, "text": text, "label": attr.get("formal_key", None),
                            "key_type": attr.get("key_type", None)}
        return out
