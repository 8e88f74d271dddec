"""io package."""
