"""Model zoo: Llama (flagship), GPT, LeNet/ResNet (vision)."""
from .llama import (LlamaConfig, LlamaForCausalLM, LlamaForCausalLMPipe, LlamaModel,  # noqa: F401
                    LlamaPretrainingCriterion, llama_flops_per_token)
from .gpt import GPTConfig, GPTForCausalLM, GPTModel, gpt_flops_per_token  # noqa: F401,E402
