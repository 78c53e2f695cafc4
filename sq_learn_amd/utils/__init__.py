"""Numerical / API substrate: validation, extmath, metrics, datasets,
model selection, tracing, checkpointing."""
