"""stages package."""
