"""Post-processor registry (config inference_settings.post_processing); the
reference ships only the abstract base (post_processing/postprocess_base.py)."""
from typing import Any, Dict


class PostProcessBase:
    @classmethod
    def _from_config(cls, config: Dict[str, Any]) -> "PostProcessBase":
        return cls(**(config or {}))

    def __call__(self, outputs):
        return outputs
