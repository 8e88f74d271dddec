"""image package."""
