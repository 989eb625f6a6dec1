"""Batch collation, resolved by name from config (data_collate: {Name: args})."""
from gnn.data_generator.data_collate.numpy_padding import BaseCollate, NumpyPadding, TypedEdgePadding  # noqa: F401
