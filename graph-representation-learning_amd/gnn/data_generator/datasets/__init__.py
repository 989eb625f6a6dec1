"""Datasets resolved by name from config (data_config.dataset.type), as in
the reference's gnn/data_generator/datasets/__init__.py.  CassiaDataset is
exported too (the reference defines it but does not export it, which breaks
its own cassia-format inference: SURVEY.md §3.2)."""
from gnn.data_generator.datasets.base_dataset import BaseDataset  # noqa: F401
from gnn.data_generator.datasets.cassia_dataset import CassiaDataset  # noqa: F401
from gnn.data_generator.datasets.datapile_dataset import DatapileDataset  # noqa: F401
