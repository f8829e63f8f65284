from .aggregation import aggregate_models, broadcast_global_model_update  # noqa: F401
