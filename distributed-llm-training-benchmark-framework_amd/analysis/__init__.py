"""dltb.analysis — metrics.csv aggregation, plots and the markdown report (reference-compatible)."""
from .make_report import generate_report  # noqa: F401
from .parse_metrics import parse_results, reference_efficiency  # noqa: F401
from .plot import plot_metrics  # noqa: F401
