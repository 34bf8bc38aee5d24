"""ORACLE TOOLING ONLY — see matplotlib/__init__.py (no attribute is used)."""
