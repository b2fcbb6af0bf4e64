"""Test stub of stable_baselines3 (see tests/stubs/README.md)."""
