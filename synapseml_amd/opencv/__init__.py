"""opencv package."""
