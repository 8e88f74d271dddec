"""featurize package."""
