"""paddle.incubate.checkpoint (reference: python/paddle/base/incubate/checkpoint/auto_checkpoint.py).

``auto_checkpoint.train_epoch_range(max_epoch_num, save_checkpoint_inter)`` iterates epochs and resumes after a
restart: the completed-epoch counter and the registered state (``register(obj)`` — Layers / optimizers /
anything with state_dict / set_state_dict) are saved under ``PADDLE_CHECKPOINT_PATH`` (or ``checkpoint_dir``) every
``save_checkpoint_inter`` seconds and at the end of each epoch that crosses the interval; on restart the loop
continues from the epoch after the last saved one, with the state restored.  The saves are atomic (write to a
temporary directory, then rename)."""
from . import auto_checkpoint  # noqa: F401

__all__ = []
