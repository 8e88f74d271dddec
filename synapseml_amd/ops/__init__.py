"""ops package."""
