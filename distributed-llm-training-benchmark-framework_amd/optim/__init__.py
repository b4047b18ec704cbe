"""dltb.optim — fused flat AdamW and DeepSpeed-compatible LR schedules."""
from .adamw import FlatAdamW  # noqa: F401
from .amp import DynamicLossScaler  # noqa: F401
from .sched import ConstantLR, WarmupLR, build_scheduler  # noqa: F401
