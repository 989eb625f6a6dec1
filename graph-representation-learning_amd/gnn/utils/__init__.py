"""Small host-side utilities the drop-in procedures need: config loading,
checkpoints, metric averaging, JSON I/O and the single-input wrapper used by
the reference's predict() (gnn/utils/*.py in the reference)."""
from gnn.utils.config import AttrDict, load_config, to_plain  # noqa: F401
from gnn.utils.json_handler import JsonHandler, read_json_file  # noqa: F401
from gnn.utils.metric_tracker import Dictlist  # noqa: F401
