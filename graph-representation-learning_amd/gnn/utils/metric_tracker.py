"""Per-key running lists with rounded means (the reference's Dictlist,
gnn/utils/metric_tracker.py:6-29): _update appends, _result averages."""
from typing import Any, Dict


class Dictlist(dict):
    def __setitem__(self, key: str, value: Any) -> None:
        self.setdefault(key, []).append(value)

    def _update(self, items: Dict[str, Any]) -> None:
        for key, value in items.items():
            self.setdefault(key, []).append(value)

    def _avg(self, key: str) -> float:
        values = self[key]
        return round(sum(values) / len(values), 3)

    def _result(self) -> Dict[str, Any]:
        return {key: self._avg(key) for key in self}
