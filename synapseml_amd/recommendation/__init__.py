"""recommendation package."""
