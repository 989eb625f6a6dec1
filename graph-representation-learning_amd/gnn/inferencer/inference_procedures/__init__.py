"""Inference procedures resolved by name from config (procedure.type)."""
from gnn.inferencer.inference_procedures.base_procedure import BaseProcedure  # noqa: F401
from gnn.inferencer.inference_procedures.kv_inference import KVInference  # noqa: F401
