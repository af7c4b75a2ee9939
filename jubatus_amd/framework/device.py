"""Device selection: one server process per MI355X.

``--gpu N`` picks the device; otherwise LOCAL_RANK (torchrun / jubavisor
launches) modulo the visible device count; ``--cpu`` or a host without a GPU
selects the host backend (NumPy oracles). On a GPU host the HIP kernel
library must load - there is no silent fallback.
"""
from __future__ import annotations

import os
from typing import Any


def gpu_available() -> bool:
    try:
        import torch
        return torch.cuda.is_available()
    except Exception:  # noqa: BLE001
        return False


def select_device(argv=None) -> Any:
    if argv is not None and getattr(argv, "cpu", False):
        return None
    if os.environ.get("JUBATUS_FORCE_CPU"):
        return None
    if not gpu_available():
        return None
    import torch
    n = torch.cuda.device_count()
    idx = getattr(argv, "gpu", None) if argv is not None else None
    if idx is None:
        idx = int(os.environ.get("LOCAL_RANK", "0")) % max(n, 1)
    torch.cuda.set_device(idx)
    from ..utils.numa import bind_to_device
    bind_to_device(idx)
    from .._native import hip_lib
    hip_lib()  # fail loudly if the kernels are missing
    return torch.device("cuda", idx)
