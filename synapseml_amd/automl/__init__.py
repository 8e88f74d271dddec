"""automl package."""
