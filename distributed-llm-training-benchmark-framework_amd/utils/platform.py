"""Platform / device facts recorded in the extended result sidecar."""
import os
import platform

import torch

# MI355X dense peaks (AMD figures with 2:1 sparsity are NOT used): docs/MI355X_HW_NOTES.md
MI355X_DENSE_BF16_FLOPS = 2.5e15
MI355X_HBM_BYTES = 288e9


def device_info(device=None) -> dict:
    info = {"host": platform.node(), "python": platform.python_version(), "torch": torch.__version__,
            "hip": getattr(torch.version, "hip", None)}
    if torch.cuda.is_available():
        idx = torch.device(device).index if device is not None and torch.device(device).index is not None else 0
        p = torch.cuda.get_device_properties(idx)
        info.update(gpu_name=p.name, gcn_arch=getattr(p, "gcnArchName", ""), cus=p.multi_processor_count,
                    hbm_gb=round(p.total_memory / 1e9, 1), visible_gpus=torch.cuda.device_count())
        try:
            info["rccl"] = ".".join(map(str, torch.cuda.nccl.version()))
        except Exception:
            pass
    for k in ("HIP_VISIBLE_DEVICES", "NCCL_MIN_NCHANNELS", "TORCH_NCCL_HIGH_PRIORITY", "HSA_ENABLE_IPC_MODE_LEGACY"):
        if k in os.environ:
            info[k] = os.environ[k]
    return info
