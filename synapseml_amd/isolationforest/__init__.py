"""isolationforest package."""
