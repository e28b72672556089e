"""Reference package `model` (model/DSTAGNN_my.py) -> dstagnn_drought_amd.model."""
