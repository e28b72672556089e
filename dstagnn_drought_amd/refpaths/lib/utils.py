"""lib/utils.py: the same names as lib/utils1.py (the reference keeps two copies)."""
from .utils1 import (cheb_polynomial, compute_val_loss_mstgcn, get_adjacency_matrix2,  # noqa: F401
                     load_graphdata_channel1, predict_and_save_results_mstgcn, re_normalization, scaled_Laplacian)
