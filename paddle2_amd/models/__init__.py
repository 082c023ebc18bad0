"""Model zoo: Llama (flagship), GPT, LeNet/ResNet (vision)."""
from .llama import (LlamaConfig, LlamaForCausalLM, LlamaForCausalLMPipe, LlamaModel,  # noqa: F401
                    LlamaPretrainingCriterion, llama_flops_per_token)
