"""dltb — an MI355X-native distributed LLM training benchmark framework.

Capabilities of deepaksatna/Distributed-LLM-Training-Benchmark-Framework
(``benchmarking/train_harness.py`` + ``scripts/``), re-designed for AMD Instinct MI355X:

* ``dltb.models``   TinyGPT (tiers A/B, reference-quirk compatible) and a Mistral-7B-shape model,
                    built from fused per-block autograd Functions whose GPU path runs
                    hand-written CDNA4 HIP kernels (``csrc/``) and hipBLASLt GEMMs.
* ``dltb.ops``      autograd-level ops over the ``dltb._C`` HIP extension (flash attention,
                    LayerNorm/RMSNorm, RoPE, GELU, softmax-xent, embedding, fused AdamW ...)
                    with bit-compatible torch reference implementations for CPU tests.
* ``dltb.parallel`` DDP (own bucketed reducer), FSDP full-shard, ZeRO-2 and ZeRO-3 engines on
                    ``torch.distributed`` (RCCL over xGMI on the GPU, gloo on the CPU).
* ``dltb.optim``    fused AdamW over flat fp32 master shards, WarmupLR, grad-norm clipping.
* ``dltb.harness``  the train_harness-compatible CLI / training loop / result export.
* ``dltb.analysis`` parse_metrics / plot / make_report (output-compatible with the reference).
"""

__version__ = "0.1.0"

from .models.config import ModelConfig, get_model_config  # noqa: F401
