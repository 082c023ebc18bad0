from . import moe  # noqa
