"""nn package."""
