"""Inference side of the drop-in API (the reference's gnn/inferencer)."""
