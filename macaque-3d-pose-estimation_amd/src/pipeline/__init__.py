"""Drop-in mirror (see src/__init__.py)."""
