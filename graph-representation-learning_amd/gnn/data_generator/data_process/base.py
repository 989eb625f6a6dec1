from typing import Any, Dict


class BaseDataProcess:
    """A sample -> sample transform built from its config args."""

    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "BaseDataProcess":
        return cls(**(config or {}))

    def __call__(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        return self.process(sample)

    def process(self, sample: Dict[str, Any]) -> Dict[str, Any]:
        raise NotImplementedError

    @staticmethod
    def ordered_lines(sample: Dict[str, Any]):
        """The sample's text lines ordered by their label index."""
        return [line for _, line in sorted(sample["label"].items(), key=lambda kv: kv[0])]
