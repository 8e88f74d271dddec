"""utils package."""
