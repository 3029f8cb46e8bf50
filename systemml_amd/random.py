"""`systemml_amd.random` — random matrix constructors of the Python DSL (reference:
src/main/python/systemml/random)."""
from .api.sampling import normal, uniform, poisson  # noqa: F401

__all__ = ["normal", "uniform", "poisson"]
