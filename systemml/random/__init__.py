"""`systemml.random` (reference: src/main/python/systemml/random)."""
from systemml_amd.api.sampling import normal, uniform, poisson  # noqa: F401

__all__ = ["normal", "uniform", "poisson"]
