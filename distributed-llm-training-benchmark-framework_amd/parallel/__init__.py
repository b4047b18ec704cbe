"""dltb.parallel — DDP, FSDP, ZeRO-2 and ZeRO-3 engines on torch.distributed (RCCL over xGMI)."""
from .checkpoint import export_consolidated, load_checkpoint, save_checkpoint  # noqa: F401
from .engine import Engine, EngineConfig  # noqa: F401
from .replicated import DDPEngine, Zero2Engine  # noqa: F401
from .graphs import GraphedStep, graphs_enabled  # noqa: F401
from .runtime import EAGER, ParamRuntime, Unit  # noqa: F401
from .sharded import FSDPEngine, Zero3Engine  # noqa: F401
from .strategy import STRATEGIES, engine_config, make_engine  # noqa: F401
