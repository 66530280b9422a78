from .metrics import compute_metrics, format_metrics, print_computed_metrics
from .linear_probe import extract_features, linear_probe
from .retrieval import embed_retrieval, evaluate_retrieval

__all__ = ["compute_metrics", "format_metrics", "print_computed_metrics", "extract_features", "linear_probe",
           "embed_retrieval", "evaluate_retrieval"]
