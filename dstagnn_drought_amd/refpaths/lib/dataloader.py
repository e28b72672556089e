"""lib/dataloader.py:5-24 (the graph loaders train_DSTAGNN_my.py:14 imports)."""
from dstagnn_drought_amd.data import load_PA, load_weighted_adjacency_matrix, load_weighted_adjacency_matrix2  # noqa: F401
