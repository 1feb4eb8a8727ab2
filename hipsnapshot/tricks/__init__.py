"""Integrations with other training stacks (DeepSpeed ZeRO-3)."""
