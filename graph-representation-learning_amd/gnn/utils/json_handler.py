"""JSON I/O with the reference's encoding convention (utf-8 with optional BOM,
gnn/utils/json_handler.py)."""
import json
from typing import Any

import numpy as np


def read_json_file(filename: str) -> Any:
    with open(filename, encoding="utf-8-sig") as f:
        return json.load(f)


class JsonHandler:
    def read_json_file(self, filename: str) -> Any:
        return read_json_file(filename)

    def dump_to_file(self, data: Any, filename: str) -> None:
        def _default(o):
            if isinstance(o, np.integer):
                return int(o)
            raise TypeError(type(o))

        with open(filename, "w", encoding="utf-8-sig") as f:
            json.dump(data, f, indent=2, ensure_ascii=False, default=_default)
