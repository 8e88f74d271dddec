"""explainers package."""
