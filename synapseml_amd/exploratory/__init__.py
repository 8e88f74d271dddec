"""exploratory package."""
