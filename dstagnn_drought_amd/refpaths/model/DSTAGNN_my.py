"""model/DSTAGNN_my.py's public names (classes :8-255, make_model :282), served by the
MI355X build: the block's compute runs in libdstagnn.so through torch.ops.dstagnn.*."""
from dstagnn_drought_amd.model import (DSTAGNN_block, DSTAGNN_submodule, Embedding, GTU,  # noqa: F401
                                       MultiHeadAttention, ScaledDotProductAttention, SMultiHeadAttention,
                                       SScaledDotProductAttention, cheb_conv, cheb_conv_withSAt, make_model)
