"""services package."""
