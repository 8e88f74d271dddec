"""cyber package."""
