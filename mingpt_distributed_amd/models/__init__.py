from .config import GPTConfig, OptimizerConfig, PRESETS
from .gpt import GPT, Block, CausalSelfAttention, MLP

__all__ = ["GPTConfig", "OptimizerConfig", "PRESETS", "GPT", "Block", "CausalSelfAttention", "MLP"]
