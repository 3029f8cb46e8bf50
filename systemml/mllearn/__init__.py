"""`systemml.mllearn` (reference: src/main/python/systemml/mllearn)."""
from systemml_amd.models.mllearn import LogisticRegression, LinearRegression, SVM, NaiveBayes  # noqa: F401
from systemml_amd.models.dl import Caffe2DML, Keras2DML  # noqa: F401

__all__ = ["LinearRegression", "LogisticRegression", "SVM", "NaiveBayes", "Caffe2DML", "Keras2DML"]
