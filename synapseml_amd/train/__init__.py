"""train package."""
