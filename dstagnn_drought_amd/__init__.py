"""dstagnn_drought_amd — MI355X-native DSTAGNN block (drop-in for Ghoul-tn/DSTAGNN_Drought's hot path).

Public surface mirrors model/DSTAGNN_my.py (make_model, DSTAGNN_block, ...) and the
graph helpers of lib/utils.py / lib/dataloader.py.  Compute runs in libdstagnn.so
(hand-written gfx950 HIP kernels behind the C-ABI in include/dstagnn.h).
"""
from .graph import (cheb_polynomial, get_adjacency_matrix2, load_PA, load_weighted_adjacency_matrix,
                    load_weighted_adjacency_matrix2, scaled_Laplacian)
from .data import load_graphdata_channel1, masked_mape_np, re_normalization, read_and_generate_dataset
from .model import (DSTAGNN_block, DSTAGNN_submodule, Embedding, GTU, MultiHeadAttention, ScaledDotProductAttention,
                    SMultiHeadAttention, SScaledDotProductAttention, cheb_conv, cheb_conv_withSAt, make_model,
                    set_direct_grads, set_dropout, set_sample_base)

__all__ = ["make_model", "DSTAGNN_block", "DSTAGNN_submodule", "cheb_conv_withSAt", "cheb_conv", "Embedding", "GTU",
           "MultiHeadAttention", "SMultiHeadAttention", "ScaledDotProductAttention", "SScaledDotProductAttention",
           "scaled_Laplacian", "cheb_polynomial", "load_weighted_adjacency_matrix", "load_weighted_adjacency_matrix2",
           "load_PA", "get_adjacency_matrix2", "load_graphdata_channel1", "read_and_generate_dataset",
           "masked_mape_np", "re_normalization", "set_dropout", "set_direct_grads", "set_sample_base"]
