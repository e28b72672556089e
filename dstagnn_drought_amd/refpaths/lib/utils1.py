"""lib/utils1.py's names used by train_DSTAGNN_my.py:15 and the model (:34-199, :294-470)."""
from dstagnn_drought_amd.data import get_adjacency_matrix2, load_graphdata_channel1, re_normalization  # noqa: F401
from dstagnn_drought_amd.graph import cheb_polynomial, scaled_Laplacian  # noqa: F401
from dstagnn_drought_amd.train import compute_val_loss_mstgcn, predict_and_save_results_mstgcn  # noqa: F401
