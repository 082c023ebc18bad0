"""paddle.callbacks (reference: python/paddle/callbacks.py)."""
from .hapi.callbacks import (Callback, EarlyStopping, LRScheduler, ModelCheckpoint, ProgBarLogger,  # noqa: F401
                             ReduceLROnPlateau, VisualDL, WandbCallback)
