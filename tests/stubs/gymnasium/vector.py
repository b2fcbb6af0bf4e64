class VectorEnv:
    """Test stub of gymnasium.vector.VectorEnv (the base class only)."""
