"""lib/metrics.py:6 masked_mape_np."""
from dstagnn_drought_amd.data import masked_mape_np  # noqa: F401
