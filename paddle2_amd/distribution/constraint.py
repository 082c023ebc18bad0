"""Constraints (reference: python/paddle/distribution/constraint.py)."""
from .variable import Constraint, Range, positive, real, simplex  # noqa: F401
from .variable import _Positive as Positive  # noqa: F401
from .variable import _Real as Real  # noqa: F401
from .variable import _Simplex as Simplex  # noqa: F401
