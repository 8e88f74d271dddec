"""dl package."""
