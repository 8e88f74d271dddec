"""vw package."""
