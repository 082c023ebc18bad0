"""Model zoo: Llama (flagship), GPT, LeNet/ResNet (vision)."""
from .llama import (LlamaConfig, LlamaForCausalLM, LlamaModel, LlamaPretrainingCriterion,  # noqa: F401
                    llama_flops_per_token)
