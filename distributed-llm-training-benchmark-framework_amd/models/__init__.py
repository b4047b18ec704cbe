"""dltb.models — TinyGPT (reference tiers) and the Mistral-7B-shape model on fused MI355X kernels."""
from .config import ModelConfig, get_model_config, TIERS  # noqa: F401


def build_model(cfg):
    """Instantiate the model family named by ``cfg.arch``."""
    if cfg.arch == "tinygpt":
        from .tinygpt import TinyGPT
        return TinyGPT(cfg)
    if cfg.arch == "mistral":
        from .mistral import MistralLM
        return MistralLM(cfg)
    raise ValueError(f"unknown arch {cfg.arch}")
