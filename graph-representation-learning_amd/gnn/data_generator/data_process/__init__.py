"""Per-sample processors, resolved by name from config (data_process: {Name: args}),
as in the reference's gnn/data_generator/data_process/__init__.py."""
from gnn.data_generator.data_process.base import BaseDataProcess  # noqa: F401
from gnn.data_generator.data_process.heuristic_graph_builder import HeuristicGraphBuilder  # noqa: F401
from gnn.data_generator.data_process.node_labeling import NodeLabeling  # noqa: F401
from gnn.data_generator.data_process.textline_encoding import TextlineEncoding  # noqa: F401
