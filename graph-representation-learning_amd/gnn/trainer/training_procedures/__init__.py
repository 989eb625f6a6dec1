"""Training procedures resolved by name from config (procedure.type), as in
the reference's gnn/trainer/training_procedures/__init__.py."""
from gnn.trainer.training_procedures.base_procedure import BaseProcedure  # noqa: F401
from gnn.trainer.training_procedures.kv_procedure import KVProcedure  # noqa: F401
