"""Model harnesses (reference: torchao/_models)."""
