from .recompute import recompute, recompute_hybrid, recompute_sequential  # noqa
