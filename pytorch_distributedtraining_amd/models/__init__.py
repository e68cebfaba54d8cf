"""Model zoo used by the benchmarks and examples (random init; no network access)."""
from .gpt2 import GPT2Block, GPT2Config, GPT2LMHeadModel, build_gpt2, gpt2_config

__all__ = ["GPT2Block", "GPT2Config", "GPT2LMHeadModel", "build_gpt2", "gpt2_config"]
