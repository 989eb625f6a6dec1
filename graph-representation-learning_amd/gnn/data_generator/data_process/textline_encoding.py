"""Node features: binary bag of characters over the charset + 4 box features
(the reference's TextlineEncoding, data_process/textline_encoding.py:10-113).

The bag uses scikit-learn's CountVectorizer(analyzer="char", binary=True) with
the charset as vocabulary -- the reference's own third-party dependency, so
lower-casing and whitespace folding behave identically."""
from __future__ import annotations

from typing import Any, Dict, List

import numpy as np

from gnn.data_generator.data_process.base import BaseDataProcess
from gnn.data_generator.data_process.normalize_text import normalize_text


class TextlineEncoding(BaseDataProcess):
    def __init__(self, is_normalized_text: bool):
        self.is_normalized_text = is_normalized_text

    def get_bow_matrix(self, textlines: List[Dict[str, Any]], char_to_idx: Dict[str, int]) -> np.ndarray:
        from sklearn.feature_extraction.text import CountVectorizer

        texts = [str(t["text"]) for t in textlines]
        if self.is_normalized_text:
            texts = [normalize_text(t) for t in texts]
        bow = CountVectorizer(vocabulary=char_to_idx, analyzer="char", binary=True).fit_transform(texts)
        return bow.toarray().astype(np.float32)

    @staticmethod
    def get_spatial_features_matrix(textlines: List[Dict[str, Any]]) -> np.ndarray:
        """(x, y, w, h) of each line's box relative to the page extent, each
        mapped v -> (v + 0.1) / 1.1 so no feature is exactly zero."""
        xs = [p[0] for t in textlines for p in t["polygon"]]
        ys = [p[1] for t in textlines for p in t["polygon"]]
        min_x, max_x, min_y, max_y = min(xs), max(xs), min(ys), max(ys)
        span_x, span_y = max_x - min_x, max_y - min_y
        out = np.zeros((len(textlines), 4), dtype=np.float64)
        for i, t in enumerate(textlines):
            px = [p[0] for p in t["polygon"]]
            py = [p[1] for p in t["polygon"]]
            x0, y0 = min(px), min(py)
            vals = ((x0 - min_x) / span_x, (y0 - min_y) / span_y, (max(px) - x0) / span_x, (max(py) - y0) / span_y)
            out[i] = [float(v + 0.1) / (0.1 + 1.0) for v in vals]
        return out.astype(np.float32)

    def process(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        if sample.get("label", None) is None:
            return sample
        lines = self.ordered_lines(sample)
        bow = self.get_bow_matrix(lines, sample["char_to_id"])
        sample["textline_encoding"] = np.concatenate((bow, self.get_spatial_features_matrix(lines)), axis=1)
        return sample
