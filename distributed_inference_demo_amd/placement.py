"""Layer-to-stage placement: the server's round-robin module arrangement, reused unchanged.

Restates `round_robin_module_arrangement` (server.py:893-903): contiguous blocks, the first
`num_modules % num_devices` devices get one extra module.  The server calls it with
(split_size, split_size) (server.py:905); this build calls it with (num_stages, n_layer),
modules := decoder layers.
"""
import numpy as np


def round_robin_module_arrangement(num_devices: int, num_modules: int) -> np.ndarray:
    arrangement = np.zeros((num_devices, num_modules), dtype=np.int64)
    per, extra = divmod(num_modules, num_devices)
    start = 0
    for i in range(num_devices):
        end = start + per + (1 if i < extra else 0)
        arrangement[i, start:end] = 1
        start = end
    return arrangement


def stage_ranges(num_stages: int, n_layer: int):
    """[(layer_begin, layer_end)] per stage from the arrangement matrix."""
    arr = round_robin_module_arrangement(num_stages, n_layer)
    out = []
    for row in arr:
        idx = np.flatnonzero(row)
        out.append((int(idx[0]), int(idx[-1]) + 1) if idx.size else (0, 0))
    return out
