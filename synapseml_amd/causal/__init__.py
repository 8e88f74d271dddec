"""causal package."""
