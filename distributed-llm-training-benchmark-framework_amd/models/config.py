"""Model configurations.

Tier table of the reference (``benchmarking/train_harness.py:157-179``):

* Tier A: vocab 32000, d 1024, 16 heads, 16 layers, block_size = seq_len  -> 236,406,784 params
* Tier B: vocab 32000, d 2048, 32 heads, 32 layers, block_size = seq_len  -> 1,681,199,104 params
  (the reference docstring calls these "1-3B" / "7-13B"; the code builds the sizes above).
* the unused TinyGPT constructor default (``train_harness.py:39-47``): d 768, 12 heads, 12 layers,
  block 4096.

Additional MI355X-era shape (not in the reference, requested by BASELINE.json config #5):

* ``M7B``: Mistral-7B shape - d 4096, 32 layers, 32 query heads / 8 KV heads (GQA), SwiGLU FFN 14336,
  RMSNorm, RoPE, causal attention, untied head, vocab 32000 (7.24B params).
"""
from dataclasses import dataclass, field, asdict
from typing import Optional


@dataclass
class ModelConfig:
    arch: str = "tinygpt"            # "tinygpt" | "mistral"
    vocab_size: int = 32000
    n_embd: int = 768
    n_head: int = 12
    n_layer: int = 12
    block_size: int = 4096
    dropout: float = 0.1
    # mistral-shape extras
    n_kv_head: Optional[int] = None
    ffn_hidden: Optional[int] = None
    rope_theta: float = 10000.0
    norm_eps: float = 1e-5
    causal: bool = False             # TinyGPT reproduces the reference's NON-causal MHA
    tie_embeddings: bool = True
    tier: str = "custom"

    @property
    def head_dim(self) -> int:
        return self.n_embd // self.n_head

    @property
    def kv_heads(self) -> int:
        return self.n_kv_head or self.n_head

    @property
    def ffn_dim(self) -> int:
        return self.ffn_hidden or 4 * self.n_embd

    def to_dict(self):
        return asdict(self)

    def num_params(self) -> int:
        """Exact parameter count (tied weights counted once), matching ``sum(p.numel())``."""
        d, V, L = self.n_embd, self.vocab_size, self.n_layer
        if self.arch == "tinygpt":
            per_block = (2 * d) + (3 * d * d + 3 * d) + (d * d + d) + (2 * d) \
                + (self.ffn_dim * d + self.ffn_dim) + (d * self.ffn_dim + d)
            return V * d + self.block_size * d + L * per_block + 2 * d
        hd = self.head_dim
        kvd = self.kv_heads * hd
        per_block = d + (d * d + 2 * kvd * d) + d * d + d + 3 * d * self.ffn_dim
        head = 0 if self.tie_embeddings else V * d
        return V * d + L * per_block + d + head

    def train_flops_per_token(self, seq_len: int) -> float:
        """6 * N_matmul + attention (12 * L * T * d non-causal, halved when causal)."""
        d, L = self.n_embd, self.n_layer
        if self.arch == "tinygpt":
            n_mat = L * (4 * d * d + 2 * d * self.ffn_dim) + self.vocab_size * d
        else:
            kvd = self.kv_heads * self.head_dim
            n_mat = L * (2 * d * d + 2 * kvd * d + 3 * d * self.ffn_dim) + self.vocab_size * d
        attn = 12 * L * seq_len * d * (0.5 if self.causal else 1.0)
        return 6.0 * n_mat + attn


TIERS = ("A", "B", "default", "M7B", "M7B_narrow", "tiny", "mtiny")


def get_model_config(tier: str, seq_len: int, dropout: float = 0.1) -> ModelConfig:
    """Reference ``get_model_config(tier, seq_len)`` plus the M7B / tiny (tests) shapes."""
    if tier == "A":
        return ModelConfig(vocab_size=32000, n_embd=1024, n_head=16, n_layer=16,
                           block_size=seq_len, dropout=dropout, tier="A")
    if tier == "B":
        return ModelConfig(vocab_size=32000, n_embd=2048, n_head=32, n_layer=32,
                           block_size=seq_len, dropout=dropout, tier="B")
    if tier == "default":
        return ModelConfig(vocab_size=32000, n_embd=768, n_head=12, n_layer=12,
                           block_size=4096, dropout=dropout, tier="default")
    if tier == "M7B":
        return ModelConfig(arch="mistral", vocab_size=32000, n_embd=4096, n_head=32, n_kv_head=8,
                           n_layer=32, ffn_hidden=14336, block_size=seq_len, dropout=0.0,
                           causal=True, tie_embeddings=False, rope_theta=10000.0, tier="M7B")
    if tier == "tiny":   # unit-test shape (CPU friendly)
        return ModelConfig(vocab_size=128, n_embd=64, n_head=4, n_layer=2, block_size=seq_len,
                           dropout=dropout, tier="tiny")
    if tier == "M7B_narrow":   # the M7B unit / collective structure (32 layers, GQA 4:1, untied head) at d 512:
        # the host-cost proxy of an eager N-rank Mistral-7B step (scripts/m7b_host_proxy.sh)
        return ModelConfig(arch="mistral", vocab_size=4096, n_embd=512, n_head=8, n_kv_head=2, n_layer=32,
                           ffn_hidden=1792, block_size=seq_len, dropout=0.0, causal=True, tie_embeddings=False,
                           rope_theta=10000.0, tier="M7B_narrow")
    if tier == "mtiny":  # Mistral-shape unit-test model: GQA 2:1, head_dim 64 (the GPU attention's smallest)
        return ModelConfig(arch="mistral", vocab_size=256, n_embd=128, n_head=2, n_kv_head=1, n_layer=2,
                           ffn_hidden=256, block_size=seq_len, dropout=0.0, causal=True,
                           tie_embeddings=False, rope_theta=10000.0, tier="mtiny")
    raise ValueError(f"Unknown tier: {tier}")
