"""Training side of the drop-in API (the reference's gnn/trainer): loss, LR
schedule and optimizer registries plus the KV training procedure."""
