"""paddle.incubate.distributed."""
from . import models  # noqa
