"""gpt-fast-style Llama decode harness (reference: torchao/_models/llama)."""
