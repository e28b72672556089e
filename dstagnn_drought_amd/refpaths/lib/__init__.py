"""Reference package `lib` (lib/dataloader.py, lib/utils.py, lib/utils1.py, lib/metrics.py)."""
